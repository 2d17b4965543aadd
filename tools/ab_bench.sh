#!/bin/bash
# A/B of extension builds on the whole benchmark: for each variants/_C.<name>.so, install it and
# run tools/bench_certify.py + bench.py (timed steps only).   bash tools/ab_bench.sh OUT v1 v2 ...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
SO=$(ls fairify_amd/_C.cpython-*.so)
for v in "$@"; do
  cp variants/_C.$v.so $SO || exit 1
  echo "== $v"
  timeout -k 10 200 python tools/bench_certify.py > $OUT/$v.cert.log 2>&1 || exit 1
  grep -h "ms" $OUT/$v.cert.log | tail -4
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --budget-pass 0 > $OUT/$v.bench.json 2> $OUT/$v.bench.err || exit 1
  python -c "import json;d=json.load(open('$OUT/$v.bench.json'));print('bench', d['ms_per_step'], d['pct_verified'])"
done
