#!/bin/bash
# Host-stream count sweep of the default N=1 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/conc
mkdir -p $O
for c in 8 6 10 8; do
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --concurrency $c --json-out $O/c$c.json > $O/c$c.txt 2>&1 || exit 1
  python -c "import json; d=json.load(open('$O/c$c.json')); print('conc $c', d['ms_per_step'], round(d['value']), d['pct_verified'], flush=True)"
done
