#!/bin/bash
# Strong-scaling emulation with the current defaults: rank r's shard of an N-rank job on one GPU.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/shards
mkdir -p $O
for sh in ${SHARDS:-0/2 0/4 0/8 7/8}; do
  tag=$(echo $sh | tr / _)
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --emulate-shard $sh --json-out $O/shard_$tag.json > $O/shard_$tag.log 2>&1
  python -c "import json; d=json.load(open('$O/shard_$tag.json')); print('$sh', d['ms_per_step'], d['value'], d['pct_verified'])"
done
