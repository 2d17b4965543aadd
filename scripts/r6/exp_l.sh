#!/bin/bash
# round 6, call L: relaxed/AC AC-7 -- what the beta fixed pass costs per setting (50 000-partition slice)
set -o pipefail
OUT=gpurun_out/r6l; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
run() {  # preset model n tag cfg
  timeout -k 10 400 python -u tools/baseline_configs.py --group $1 --models $2 --max-partitions $3 \
    --out $OUT/$4 --cfg "$5" > $OUT/$4.log 2>&1 || { tail -30 $OUT/$4.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$4/${1//\//_}/summary.json'))
for r in d['models']: print('$4', r['model'], 'unk', r['UNK'], 'cov', r['Cov_sound%'], 'wall', r['wall_s'], r.get('stage_nodes'), {k: v for k, v in r.get('stage_s', {}).items() if k in ('bab', 'beta', 'relu')})"
}
run relaxed/AC AC-7 50000 def ""
run relaxed/AC AC-7 50000 it64 "beta_iters=64"
run relaxed/AC AC-7 50000 probe4 "beta_probe_levels=4"
run relaxed/AC AC-7 50000 b64 "beta_budget=64"
run relaxed/AC AC-7 50000 k64 "beta_branch=kernel,beta_iters=64"
run relaxed/AC AC-7 50000 k64_p4 "beta_branch=kernel,beta_iters=64,beta_probe_levels=4"
