#!/bin/bash
# round 6, call A: beta kernel tests (pgap, orientation sign, relaxed GPU twins), BM-8 residue
# branching / orientation A/B, one default bench for this lease
set -o pipefail
OUT=gpurun_out/r6a; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
true
true
S="--set sep_b1024:node_budget=1024,merge_orient=0"
S="$S --set k_b1024:node_budget=1024"
S="$S --set pg0_b1024:branch=pgap,lookahead=0,node_budget=1024"
S="$S --set pg8_b1024:branch=pgap,lookahead=8,node_budget=1024"
S="$S --set pg0_b4096:branch=pgap,lookahead=0,node_budget=4096"
S="$S --set pg8_b4096:branch=pgap,lookahead=8,node_budget=4096"
timeout -k 10 600 python -u tools/exp/beta_residue.py --npz tools/exp/data/relaxedBM_BM-8_unknown.npz --n 200 $S > $OUT/res_bm8.log 2>&1 || { tail -30 $OUT/res_bm8.log; exit 1; }
cat $OUT/res_bm8.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --budget-pass 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
