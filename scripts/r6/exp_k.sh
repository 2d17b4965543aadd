#!/bin/bash
# round 6, call K: relaxed/BM BM-8 full grid, the infeasibility pass on / off at the fixed-pass budget
set -o pipefail
OUT=gpurun_out/r6k; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
run() {  # preset model n tag cfg
  timeout -k 10 400 python -u tools/baseline_configs.py --group $1 --models $2 --max-partitions $3 \
    --out $OUT/$4 --cfg "$5" > $OUT/$4.log 2>&1 || { tail -30 $OUT/$4.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$4/${1//\//_}/summary.json'))
for r in d['models']: print('$4', r['model'], 'unk', r['UNK'], 'cov', r['Cov_sound%'], 'wall', r['wall_s'], r.get('stage_nodes'), {k: v for k, v in r.get('stage_s', {}).items() if k in ('bab', 'beta', 'relu')})"
}
run relaxed/BM BM-8 2000000 f0 "beta_feas_iters=0"
run relaxed/BM BM-8 2000000 f64 "beta_feas_iters=64"
run relaxed/BM BM-8 2000000 f0_it64 "beta_feas_iters=0,beta_iters=64"
