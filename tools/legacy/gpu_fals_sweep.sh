#!/bin/bash
# Residual falsifier cost/benefit at the current defaults (full bench, and the 1/8 shard).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/fals
mkdir -p $O
run() {
  tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --json-out $O/$tag.json > $O/$tag.log 2>&1
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', '$*', d['ms_per_step'], d['value'], d['pct_verified'])"
}
run off --residual-samples 0
run it8 --residual-iters 8
run it0 --residual-iters 0
run s8_def --emulate-shard 0/8 --steps 2
run s8_off --emulate-shard 0/8 --steps 2 --residual-samples 0
run s8_it8 --emulate-shard 0/8 --steps 2 --residual-iters 8
