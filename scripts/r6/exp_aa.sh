#!/bin/bash
# round 6, call AA: run-to-run identity after the race fix -- relaxed/BM BM-4 + BM-8 and stress/BM BM-8,
# twice each (before the fix 2 of 3 multi-threaded runs differed)
set -o pipefail
OUT=gpurun_out/r6aa; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python -u tools/baseline_configs.py --group relaxed/BM --models BM-4,BM-8 --out $OUT/rbm_$i > $OUT/rbm_$i.log 2>&1 || { tail -30 $OUT/rbm_$i.log; exit 1; }
  grep "(zoo)" $OUT/rbm_$i.log
  timeout -k 10 200 python -u tools/baseline_configs.py --group stress/BM --models BM-8 --out $OUT/sbm_$i > $OUT/sbm_$i.log 2>&1 || { tail -30 $OUT/sbm_$i.log; exit 1; }
  grep "(zoo)" $OUT/sbm_$i.log
done
