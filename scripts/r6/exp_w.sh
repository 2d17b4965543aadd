#!/bin/bash
# round 6, call W: the native beta loop with UNSAT only on all-trees-closed evidence (unclosed, dev_next stats)
set -o pipefail
OUT=gpurun_out/r6w; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_beta_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
export PYTHONFAULTHANDLER=1
for i in 1 2; do
  FAIRIFY_BETA_LOG=1 timeout -k 10 300 python -u tools/baseline_configs.py --group relaxed/BM --models BM-4 \
    --out $OUT/bm4_$i > $OUT/bm4_$i.log 2>&1 || { tail -30 $OUT/bm4_$i.log; exit 1; }
  grep "BM-4 (zoo)" $OUT/bm4_$i.log
  grep -o "unclosed.: [0-9]*\|dev_next.: [0-9]*" $OUT/bm4_$i.log | head -5 || true
done
