#!/bin/bash
# round 6, call F: beta fixed-pass settings (branch x steps, sign-pruned roots) on AC-7 slices and the
# full relaxed/BM BM-8 grid; GPU tests of the beta / relu stages first
set -o pipefail
OUT=gpurun_out/r6f; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
timeout -k 10 600 python -u -m pytest tests/test_beta_gpu.py tests/test_relu_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
run() {  # preset model n tag cfg
  timeout -k 10 400 python -u tools/baseline_configs.py --group $1 --models $2 --max-partitions $3 \
    --out $OUT/$4 --cfg "$5" > $OUT/$4.log 2>&1 || { tail -30 $OUT/$4.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$4/${1//\//_}/summary.json'))
for r in d['models']: print('$4', r['model'], 'unk', r['UNK'], 'cov', r['Cov_sound%'], 'wall', r['wall_s'], r.get('stage_nodes'), {k: v for k, v in r.get('stage_s', {}).items() if k in ('bab', 'beta', 'relu')})"
}
run relaxed/AC AC-7 50000 r_k64 "beta_branch=kernel,beta_iters=64"
run relaxed/AC AC-7 50000 r_p64 "beta_branch=pgap,beta_iters=64"
run relaxed/AC AC-7 50000 r_p128 ""
run relaxed/AC AC-7 50000 r_nobeta "beta_budget=0"
run stress/AC AC-7 200000 s_p64 "beta_branch=pgap,beta_iters=64"
run relaxed/BM BM-8 2000000 bm8_k64 "beta_branch=kernel,beta_iters=64"
run relaxed/BM BM-8 2000000 bm8_p64 "beta_branch=pgap,beta_iters=64"
run relaxed/BM BM-8 2000000 bm8_p128 ""
