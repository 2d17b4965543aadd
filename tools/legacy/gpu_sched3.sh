#!/bin/bash
# Level-start budget rule: first-pass budget x escalation filter sweep (bench default suite).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/sched3
mkdir -p $O
for nb in ${NBS:-192 256 384}; do
  for mo in ${MOS:-64 128 192}; do
    tag=nb${nb}_mo${mo}
    timeout -k 10 300 python bench.py --node-budget $nb --escalate-max-open $mo --json-out $O/$tag.json > $O/$tag.log 2>&1
    python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['pct_verified'])"
  done
done
