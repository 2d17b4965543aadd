#!/bin/bash
# Per-model pipeline diagnostic + rocprofv3 kernel stats of the default bench.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 python tools/diag_models.py --json-out gpurun_out/diag_models.json "$@" > gpurun_out/diag.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 1 --warmup 0 > gpurun_out/prof/bench_stdout.txt 2>&1
find gpurun_out/prof -name "*stats*"
