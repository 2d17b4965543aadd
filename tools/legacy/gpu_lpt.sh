#!/bin/bash
# LPT item ordering (measured item times of the previous step) at the full suite and shards.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/lpt
mkdir -p $O
run() {
  tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --json-out $O/$tag.json > $O/$tag.log 2>&1
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', '$*', d['ms_per_step'], d['value'], d['pct_verified'])"
}
run full --steps 2
run s8 --emulate-shard 0/8 --steps 3
run s8b --emulate-shard 7/8 --steps 3
run s4 --emulate-shard 0/4 --steps 3
run s2 --emulate-shard 1/2 --steps 2
