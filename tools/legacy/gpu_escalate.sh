#!/bin/bash
# Bench sweep of the escalated second BaB pass (node budget of the residue pass).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/escalate
for e in ${ESC_LIST:-0 8192 16384 32768}; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --escalate-budget $e --json-out gpurun_out/escalate/e$e.json \
    > gpurun_out/escalate/e$e.log 2>&1
  tail -1 gpurun_out/escalate/e$e.log
done
