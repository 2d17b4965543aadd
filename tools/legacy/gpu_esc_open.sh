#!/bin/bash
# Escalation-filter sweep after the deterministic open-frontier count (open inner nodes of the
# level where the budget ran out).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/esc_open
mkdir -p $O
for mo in ${MOS:-48 96 128 192}; do
  timeout -k 10 300 python bench.py --escalate-max-open $mo --json-out $O/mo_$mo.json > $O/mo_$mo.log 2>&1
  python -c "import json; d=json.load(open('$O/mo_$mo.json')); print('max_open $mo', d['ms_per_step'], d['value'], d['pct_verified'])"
done
