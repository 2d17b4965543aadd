#!/bin/bash
# BaB runtime / bench-structure changes: GPU tests, default bench, variants, trace busy fraction.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof3
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --json-out gpurun_out/bench_c8.json
timeout -k 10 600 python bench.py --chunk 2048 --json-out gpurun_out/bench_c8_2048.json
timeout -k 10 600 python bench.py --concurrency 4 --json-out gpurun_out/bench_c4.json
timeout -k 10 600 python bench.py --emulate-shard 0/8 --json-out gpurun_out/bench_shard8.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o bench -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof3/bench_stdout.txt 2>&1
python tools/trace_busy.py gpurun_out/prof3/bench_kernel_trace.csv
