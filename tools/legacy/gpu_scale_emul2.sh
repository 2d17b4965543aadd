#!/bin/bash
# Strong-scaling emulation (one rank's shard of an N-rank job on one GPU) with the bench defaults.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/scale2
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --json-out gpurun_out/scale2/n1.json > gpurun_out/scale2/n1.log 2>&1
python -c "import json; d=json.load(open('gpurun_out/scale2/n1.json')); print('1/1', d['ms_per_step'], d['value'], d['pct_verified'])"
for sh in 0/2 1/2 0/4 3/4 0/8 5/8 7/8; do
  tag=$(echo $sh | tr / _)
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --emulate-shard $sh --json-out gpurun_out/scale2/$tag.json > gpurun_out/scale2/$tag.log 2>&1
  python -c "import json; d=json.load(open('gpurun_out/scale2/$tag.json')); print('$sh', d['ms_per_step'], d['value'], d['pct_verified'])"
done
