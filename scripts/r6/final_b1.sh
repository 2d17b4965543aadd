#!/bin/bash
# round 6 final one-HEAD baseline, call 1: the race-fix check (relaxed/BM BM-4 with the beta log), then
# stress and targeted (GPU stages only)
set -o pipefail
OUT=gpurun_out/r6fin; mkdir -p $OUT
FAIRIFY_BETA_LOG=1 timeout -k 10 300 python -u tools/baseline_configs.py --group relaxed/BM --models BM-4 \
  --out $OUT/bm4_check > $OUT/bm4_check.log 2>&1 || { tail -30 $OUT/bm4_check.log; exit 1; }
grep "BM-4 (zoo)" $OUT/bm4_check.log
export BASE_OUT=$OUT
TLIM=500 bash scripts/r6/base.sh stress && TLIM=300 bash scripts/r6/base.sh targeted
