#!/bin/bash
# round 6, call T: NaN-safe node closure in the native beta loop (a NaN bound used to count as closed);
# relaxed/BM BM-4 twice with the beta stage log (nan_nodes per chunk), GPU beta tests
set -o pipefail
OUT=gpurun_out/r6t; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
timeout -k 10 300 python -u -m pytest tests/test_beta_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  FAIRIFY_BETA_LOG=1 timeout -k 10 300 python -u tools/baseline_configs.py --group relaxed/BM --models BM-4 \
    --out $OUT/bm4_$i > $OUT/bm4_$i.log 2>&1 || { tail -30 $OUT/bm4_$i.log; exit 1; }
  grep "BM-4 (zoo)" $OUT/bm4_$i.log
  grep -c "nan_nodes" $OUT/bm4_$i.log || true
done
