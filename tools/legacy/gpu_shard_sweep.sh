#!/bin/bash
# 1/8-shard sweep of item size and host concurrency at the current defaults (one GPU).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/shard_sweep
mkdir -p $O
run() {
  tag=$1; shift
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --json-out $O/$tag.json "$@" > $O/$tag.txt 2>&1 || return 1
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], round(d['value']), d['pct_verified'], flush=True)"
}
run s08_c4096 --emulate-shard 0/8 &&
run s08_c2000 --emulate-shard 0/8 --chunk 2000 &&
run s08_c1000 --emulate-shard 0/8 --chunk 1000 &&
run s08_c4096_t12 --emulate-shard 0/8 --concurrency 12 &&
run s78_c4096 --emulate-shard 7/8 &&
run s78_c1000 --emulate-shard 7/8 --chunk 1000
