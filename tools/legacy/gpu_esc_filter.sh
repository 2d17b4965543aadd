#!/bin/bash
# Bench sweep: escalated residue pass with the open-frontier filter.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/escf
for spec in 8192:512 16384:512 16384:768 32768:512 8192:0; do
  e=${spec%%:*}; o=${spec##*:}
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --escalate-budget $e --escalate-max-open $o \
    --json-out gpurun_out/escf/e${e}_o${o}.json > gpurun_out/escf/e${e}_o${o}.log 2>&1
  python -c "import json; d=json.load(open('gpurun_out/escf/e${e}_o${o}.json')); print('e=$e o=$o', d['ms_per_step'], d['value'], d['pct_verified'])"
done
