#!/bin/bash
# Micro-benchmark A/B of extension builds: for each variants/_C.<name>.so, install it as the
# in-tree extension and run tools/bench_bounds.py on MODELS.   bash tools/ab_micro.sh OUT MODELS v1 v2 ...
set -o pipefail
OUT=gpurun_out/$1; shift
MODELS=$1; shift
mkdir -p $OUT
SO=$(ls fairify_amd/_C.cpython-*.so)
for v in "$@"; do
  cp variants/_C.$v.so $SO || exit 1
  echo "== $v"
  timeout -k 10 200 python tools/bench_bounds.py --models $MODELS --rows 131072 --iters 20 > $OUT/$v.log 2>&1 || exit 1
  grep -h model $OUT/$v.log | python -c "import sys,json;[print(d['model'], d['ms']) for d in map(json.loads, sys.stdin)]"
done
