#!/bin/bash
# Bench sweep over BaB budget schedules: first-pass budget, then escalation stages
# (budget:max_open), each on the residue whose open frontier stayed small.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/sched
i=0
for spec in ${SCHED:-"2048|16384|768|"}; do
  IFS='|' read nb eb eo st <<< "$spec"
  i=$((i+1)); tag=$(echo "$spec" | tr "|:" "__")
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --node-budget $nb --escalate-budget $eb --escalate-max-open $eo \
    ${st:+--stages $st} --json-out gpurun_out/sched/$tag.json > gpurun_out/sched/$tag.log 2>&1
  python -c "import json; d=json.load(open('gpurun_out/sched/$tag.json')); print('$spec', d['ms_per_step'], d['value'], d['pct_verified'])"
done
