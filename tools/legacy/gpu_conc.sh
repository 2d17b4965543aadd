#!/bin/bash
# Host-thread / stream concurrency at the full suite and the 1/8 shard.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/conc
mkdir -p $O
run() {
  tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --json-out $O/$tag.json > $O/$tag.log 2>&1
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', '$*', d['ms_per_step'], d['value'], d['pct_verified'])"
}
for c in 8 12 16; do
  run s8_c$c --emulate-shard 0/8 --steps 3 --concurrency $c
done
for c in 6 12; do
  run full_c$c --steps 2 --concurrency $c
done
run s8_c12_ch1000 --emulate-shard 0/8 --steps 3 --concurrency 12 --chunk 1000
