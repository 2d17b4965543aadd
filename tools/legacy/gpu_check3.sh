#!/bin/bash
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -80 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --scope chunk --chunk 4096 --steps 1 --warmup 1 --concurrency 1 | tee gpurun_out/bench_c1.json
timeout -k 10 600 python bench.py --scope chunk --chunk 4096 --steps 1 --warmup 1 --concurrency 4 | tee gpurun_out/bench_c4.json
timeout -k 10 900 python bench.py | tee gpurun_out/bench_default.json
