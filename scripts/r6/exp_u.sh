#!/bin/bash
# round 6, call U: cross-stream hazard hunt -- root bounds (be.bounds symbolic + refine + crown) from 4
# host threads vs serial (BM-4, AC-7); relaxed/BM BM-4 with the crossed-bounds guard (beta log)
set -o pipefail
OUT=gpurun_out/r6u; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
timeout -k 10 300 python -u -m pytest tests/test_beta_gpu.py -x -q -k "crossed or bruteforce" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u tools/exp/bounds_concurrency.py --model BM-4 --rows 3000 --threads 4 --reps 5 > $OUT/conc_bm4.log 2>&1 || { tail -30 $OUT/conc_bm4.log; exit 1; }
grep -v Warn $OUT/conc_bm4.log
timeout -k 10 300 python -u tools/exp/bounds_concurrency.py --model AC-7 --preset stress/AC --rows 3000 --threads 4 --reps 3 > $OUT/conc_ac7.log 2>&1 || { tail -30 $OUT/conc_ac7.log; exit 1; }
grep -v Warn $OUT/conc_ac7.log
for i in 1 2; do
  FAIRIFY_BETA_LOG=1 timeout -k 10 300 python -u tools/baseline_configs.py --group relaxed/BM --models BM-4 \
    --out $OUT/bm4_$i > $OUT/bm4_$i.log 2>&1 || { tail -30 $OUT/bm4_$i.log; exit 1; }
  grep "BM-4 (zoo)" $OUT/bm4_$i.log
done
