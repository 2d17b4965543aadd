#!/bin/bash
# round 6, call O: the beta fixed pass on BM-4 (150-wide: weights from L2, 7 waves per CU) -- the
# 128-width cap lifted, relaxed/BM and targeted2/BM BM-4 full grids
set -o pipefail
OUT=gpurun_out/r6o; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
timeout -k 10 300 python -u -m pytest tests/test_beta_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
run() {  # preset model n tag cfg
  timeout -k 10 400 python -u tools/baseline_configs.py --group $1 --models $2 --max-partitions $3 \
    --out $OUT/$4 --cfg "$5" > $OUT/$4.log 2>&1 || { tail -30 $OUT/$4.log; exit 1; }
  python -c "
import json, glob; d=json.load(open(glob.glob('$OUT/$4/*/summary.json')[0]))
for r in d['models']: print('$4', r['model'], 'unk', r['UNK'], 'cov', r['Cov_sound%'], 'wall', r['wall_s'], r.get('stage_nodes'), {k: v for k, v in r.get('stage_s', {}).items() if k in ('bab', 'beta', 'relu')})"
}
run relaxed/BM BM-4 2000000 bm4_w256 "beta_max_width=256"
run targeted2/BM BM-4 2000000 t2bm4_w256 "beta_max_width=256"
run relaxed/AC AC-7 50000 r7_def ""
run relaxed/AC AC-7 50000 r7_cap2k "beta_escalate_cap=2048"
run relaxed/AC AC-7 50000 r7_cap4k "beta_escalate_cap=4096"
