#!/bin/bash
# rocprofv3 kernel stats of the default bench (with the escalated residue pass).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_esc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_esc -o run -- python3 bench.py --steps 1 --warmup 1 --concurrency 4 \
  > gpurun_out/prof_esc/bench.log 2>&1
tail -1 gpurun_out/prof_esc/bench.log
find gpurun_out/prof_esc -name "*kernel_stats.csv" | head -3
python tools/trace_busy.py gpurun_out/prof_esc/run_kernel_trace.csv || true
rm -f gpurun_out/prof_esc/run_kernel_trace.csv
head -25 gpurun_out/prof_esc/run_kernel_stats.csv | cut -d, -f1-5
