#!/bin/bash
# round 6, call H: beta optimisation depth (decay / steps) x the infeasibility pass, on the BM-8 residue
# and the AC-7 / BM-8 big-grid rows
set -o pipefail
OUT=gpurun_out/r6h; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
timeout -k 10 600 python -u -m pytest tests/test_beta_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
B="node_budget=1024"
S="--set f0:$B,feas_iters=0"
S="$S --set f64:$B,feas_iters=64"
S="$S --set d995_f0:$B,feas_iters=0,decay=0.995,iters=256,root_iters=800"
S="$S --set d995_f64:$B,feas_iters=64,decay=0.995,iters=256,root_iters=800"
S="$S --set d995_f128:$B,feas_iters=128,decay=0.995,iters=256,root_iters=800"
S="$S --set d995_f64_b4096:node_budget=4096,feas_iters=64,decay=0.995,iters=256,root_iters=800"
timeout -k 10 800 python -u tools/exp/beta_residue.py --npz tools/exp/data/relaxedBM_BM-8_unknown.npz --n 200 $S > $OUT/res_bm8.log 2>&1 || { tail -30 $OUT/res_bm8.log; exit 1; }
cat $OUT/res_bm8.log
run() {  # preset model n tag cfg
  timeout -k 10 400 python -u tools/baseline_configs.py --group $1 --models $2 --max-partitions $3 \
    --out $OUT/$4 --cfg "$5" > $OUT/$4.log 2>&1 || { tail -30 $OUT/$4.log; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/$4/${1//\//_}/summary.json'))
for r in d['models']: print('$4', r['model'], 'unk', r['UNK'], 'cov', r['Cov_sound%'], 'wall', r['wall_s'], r.get('stage_nodes'), {k: v for k, v in r.get('stage_s', {}).items() if k in ('bab', 'beta', 'relu')})"
}
run relaxed/BM BM-8 2000000 bm8_f64 "beta_feas_iters=64"
run relaxed/BM BM-8 2000000 bm8_d995_f64 "beta_feas_iters=64,beta_decay=0.995,beta_iters=256"
run stress/AC AC-7 200000 s_f64 "beta_feas_iters=64"
run relaxed/AC AC-7 50000 r_k64_f64 "beta_branch=kernel,beta_iters=64,beta_feas_iters=64"
run relaxed/AC AC-7 50000 r_f64 "beta_feas_iters=64"
