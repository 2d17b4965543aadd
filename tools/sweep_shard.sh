#!/bin/bash
# 1/8-shard schedule sweep: bench.py --emulate-shard 0/8 with each "_"-separated extra-argument
# set (one per line in the output).   bash tools/sweep_shard.sh OUT "ARGS1" "ARGS2" ...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
n=0
for a in "$@"; do
  n=$((n+1))
  timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --budget-pass 0 --emulate-shard 0/8 ${a//_/ } > $OUT/s$n.json 2> $OUT/s$n.err || exit 1
  python -c "import json;d=json.load(open('$OUT/s$n.json'));print('$a', d['ms_per_step'], d['pct_verified'])"
done
