#!/bin/bash
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -80 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 900 python bench.py --profile --scope chunk --chunk 4096 --steps 1 --warmup 1 2> gpurun_out/bench_profile.txt | tee gpurun_out/bench.json
tail -25 gpurun_out/bench_profile.txt
