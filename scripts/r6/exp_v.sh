#!/bin/bash
# round 6, call V: whole-chunk beta decisions at the root level (exp T/U) -- root-level skip diagnostics of
# the native loop (not RUNNING / relaxed-dead), and the torch loop on the same run
set -o pipefail
OUT=gpurun_out/r6v; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
for i in 1 2 t; do
  env_t=""; [ "$i" = "t" ] && export FAIRIFY_TORCH_BETA=1
  FAIRIFY_BETA_LOG=1 timeout -k 10 300 python -u tools/baseline_configs.py --group relaxed/BM --models BM-4 \
    --out $OUT/bm4_$i > $OUT/bm4_$i.log 2>&1 || { tail -30 $OUT/bm4_$i.log; exit 1; }
  grep "BM-4 (zoo)" $OUT/bm4_$i.log
  grep "root_skip" $OUT/bm4_$i.log | head -5 || true
done
