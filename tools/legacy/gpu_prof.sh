#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (summaries copied to profiles/ by hand).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --scope chunk --chunk 4096 --steps 1 --warmup 0 "$@" > gpurun_out/prof/bench_stdout.txt 2>&1
find gpurun_out/prof -name "*stats*" | head
