#!/bin/bash
# round 6, call Q: beta weight placement bitwise test; relaxed/BM BM-4 twice with the beta stage log
# (the round-end run decided 302 partitions in beta, the exp O run at the same settings 2 586)
set -o pipefail
OUT=gpurun_out/r6q; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
timeout -k 10 300 python -u -m pytest tests/test_beta_gpu.py -x -q -k "placement or bruteforce" --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  FAIRIFY_BETA_LOG=1 timeout -k 10 300 python -u tools/baseline_configs.py --group relaxed/BM --models BM-4 \
    --out $OUT/bm4_$i > $OUT/bm4_$i.log 2>&1 || { tail -30 $OUT/bm4_$i.log; exit 1; }
  grep "BM-4 (zoo)" $OUT/bm4_$i.log
  grep "^\[beta\]" $OUT/bm4_$i.log | head -5
done
