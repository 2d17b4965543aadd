#!/bin/bash
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof4
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --json-out gpurun_out/bench_c8.json
timeout -k 10 600 python bench.py --profile --json-out gpurun_out/bench_prof.json 2> gpurun_out/bench_profile.txt
tail -22 gpurun_out/bench_profile.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4 -o bench -- python3 bench.py --steps 1 --warmup 1 --concurrency 4 > gpurun_out/prof4/bench_stdout.txt 2>&1
python tools/trace_busy.py gpurun_out/prof4/bench_kernel_trace.csv
rm -f gpurun_out/prof4/bench_kernel_trace.csv
