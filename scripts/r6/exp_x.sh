#!/bin/bash
# round 6, call X: diagnostics of beta groups closed whole at the root level (FAIRIFY_BETA_CHECK): the pool's
# root arrays and the same roots through the torch loop's kernel call
set -o pipefail
OUT=gpurun_out/r6x; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
for i in 1 2; do
  FAIRIFY_BETA_CHECK=1 FAIRIFY_BETA_LOG=1 timeout -k 10 300 python -u tools/baseline_configs.py --group relaxed/BM \
    --models BM-4 --out $OUT/bm4_$i > $OUT/bm4_$i.log 2>&1 || { tail -30 $OUT/bm4_$i.log; exit 1; }
  grep "BM-4 (zoo)" $OUT/bm4_$i.log
  grep "beta-check" $OUT/bm4_$i.log | head -6 | cut -c1-400 || true
done
