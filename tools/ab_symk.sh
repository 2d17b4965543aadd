#!/bin/bash
# Same-lease A/B of the symbolic bound kernel: HEAD vs a pre-change tree built in ab_pre/
# (git archive <sha> | tar -x -C ab_pre; build there).  Alternating timed runs of
# tools/bench_bounds.py, then one PMC pass (LDS instructions / bank conflicts / wave cycles) per tree.
#   bash tools/ab_symk.sh OUT MODELS ROWS
set -o pipefail
OUT=gpurun_out/$1; MODELS=${2:-AC-7,AC-4,AC-1}; ROWS=${3:-131072}
R=$(pwd)
mkdir -p $OUT
for rep in 1 2; do
  for tree in head pre; do
    d=$R; [ $tree = pre ] && d=$R/ab_pre
    (cd $d && timeout -k 10 300 python -u tools/bench_bounds.py --models $MODELS --rows $ROWS --mode symbolic \
      --iters 20 --json-out $R/$OUT/$tree.$rep.json > $R/$OUT/$tree.$rep.log 2>&1) || exit $?
    echo "[ab_symk] $tree rep $rep done"
  done
done
for tree in head pre; do
  d=$R; [ $tree = pre ] && d=$R/ab_pre
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS \
     SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_MFMA --output-format csv \
     -d $R/$OUT/pmc_$tree -o run -- python3 $d/tools/bench_bounds.py --models $MODELS --rows $ROWS --mode symbolic \
     --iters 3 > $R/$OUT/pmc_$tree.log 2>&1) || exit $?
  echo "[ab_symk] pmc $tree done"
done
