#!/bin/bash
# A/B of extension builds on the GPU box: for each variants/_C.<name>.so, install it as the
# in-tree extension and run the crown/certify micro-benchmarks and a short bench.py.
#   bash tools/ab_variants.sh OUT name1 name2 ...
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
SO=$(ls fairify_amd/_C.cpython-*.so)
for v in "$@"; do
  cp variants/_C.$v.so $SO || exit 1
  timeout -k 10 200 python tools/bench_crown.py --iters 10 > $OUT/$v.crown.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --budget-pass 0 > $OUT/$v.bench.json 2> $OUT/$v.bench.err || exit 1
  echo "== $v"; grep -h "model\|ms" $OUT/$v.crown.log | tail -6; python -c "import json;d=json.load(open('$OUT/$v.bench.json'));print('bench ms/step',d['ms_per_step'],'pct',d['pct_verified'])"
done
