#!/bin/bash
# round 6, call S: run-to-run differences of the beta fixed pass on relaxed/BM BM-4 (exp Q: 9 024 vs
# 6 811 UNKNOWN on two consecutive runs of the same tree), bisected by toggles
set -o pipefail
OUT=gpurun_out/r6s; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
timeout -k 10 500 python -u tools/exp/beta_determinism.py --preset relaxed/BM --model BM-4 --limit 200000 --settings nat,nat --threads 4 \
  > $OUT/det_bm4.log 2>&1 || { tail -30 $OUT/det_bm4.log; exit 1; }
cat $OUT/det_bm4.log | grep -v Warning
