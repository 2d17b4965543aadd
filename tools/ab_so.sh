#!/bin/bash
# A/B of extension builds on the whole benchmark, alternating:  bash tools/ab_so.sh OUT DIR v1 v2 ...
# Each DIR/_C.<v>.so is copied over the in-tree extension (of the box's snapshot) before a
# bench.py run (3 timed steps, no budget pass).  Build variants with
#   FAIRIFY_HIPCC_DEFINES="MACRO=VALUE" python -m fairify_amd.csrc.build --out DIR/_C.<v>.so --tag <v>
set -o pipefail
OUT=gpurun_out/$1; shift
DIR=$1; shift
mkdir -p $OUT
SO=$(ls fairify_amd/_C.cpython-*.so)
n=0
for v in "$@"; do
  n=$((n+1))
  cp $DIR/_C.$v.so $SO || exit 1
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --budget-pass 0 > $OUT/$v.$n.json 2> $OUT/$v.$n.err || exit 1
  python -c "import json;d=json.load(open('$OUT/$v.$n.json'));print('$v', d['ms_per_step'], d['pct_verified'])"
done
