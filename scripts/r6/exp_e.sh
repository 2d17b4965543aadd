#!/bin/bash
# round 6, call E: BM-8 residue -- convergence of the children's optimisation under pgap (decay,
# child step size), look-ahead width, budgets
set -o pipefail
OUT=gpurun_out/r6e; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
B="node_budget=1024"
S="--set base:$B"
S="$S --set dec99:$B,decay=0.99"
S="$S --set dec995_it256:$B,decay=0.995,iters=256,root_iters=800"
S="$S --set clr06:$B,child_lr=0.6"
S="$S --set clr1:$B,child_lr=1.0"
S="$S --set la0:$B,lookahead=0"
S="$S --set la4:$B,lookahead=4"
S="$S --set nowarm:$B,warm_beta=0"
S="$S --set b2048:node_budget=2048"
S="$S --set b4096:node_budget=4096"
timeout -k 10 800 python -u tools/exp/beta_residue.py --npz tools/exp/data/relaxedBM_BM-8_unknown.npz --n 200 $S > $OUT/res_bm8.log 2>&1 || { tail -30 $OUT/res_bm8.log; exit 1; }
cat $OUT/res_bm8.log
