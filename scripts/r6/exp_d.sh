#!/bin/bash
# round 6, call D: GPU tests of the touched stages; AC-7 slices of stress/AC and relaxed/AC with the
# beta stage's new defaults (pgap, 128 steps) and input-split escalation caps / beta budgets
set -o pipefail
OUT=gpurun_out/r6d; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
timeout -k 10 600 python -u -m pytest tests/test_beta_gpu.py tests/test_relu_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
run() {  # preset n tag cfg
  timeout -k 10 400 python -u tools/baseline_configs.py --group $1 --models AC-7 --max-partitions $2 \
    --out $OUT/$3 --cfg "$4" > $OUT/$3.log 2>&1 || { tail -30 $OUT/$3.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$3/${1//\//_}/summary.json'))
for r in d['models']: print('$3', r['model'], 'unk', r['UNK'], 'wall', r['wall_s'], r.get('stage_nodes'), {k: v for k, v in r.get('stage_s', {}).items() if k in ('bab', 'beta', 'beta.native')})"
}
run stress/AC 200000 s_def ""
run stress/AC 200000 s_kern "beta_branch=kernel,beta_iters=64"
run stress/AC 200000 s_cap2k "beta_escalate_cap=2048"
run stress/AC 200000 s_cap2k_b256 "beta_escalate_cap=2048,beta_budget=256"
run stress/AC 200000 s_cap4k_b256 "beta_escalate_cap=4096,beta_budget=256"
run relaxed/AC 50000 r_def ""
run relaxed/AC 50000 r_kern "beta_branch=kernel,beta_iters=64"
run relaxed/AC 50000 r_cap2k "beta_escalate_cap=2048"
