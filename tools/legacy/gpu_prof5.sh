#!/bin/bash
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof5
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5 -o bench -- python3 bench.py --steps 1 --warmup 1 --concurrency 4 > gpurun_out/prof5/bench_stdout.txt 2>&1
python tools/trace_busy.py gpurun_out/prof5/bench_kernel_trace.csv
rm -f gpurun_out/prof5/bench_kernel_trace.csv
head -25 gpurun_out/prof5/bench_kernel_stats.csv | cut -d, -f1-5
