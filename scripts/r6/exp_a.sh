#!/bin/bash
# round 6, call A: beta kernel tests (pgap + relaxed GPU twins), BM-8 residue branching A/B,
# one default bench for this lease
set -o pipefail
OUT=gpurun_out/r6a; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
timeout -k 10 600 python -u -m pytest tests/test_beta_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/tests_beta.log 2>&1 || { tail -30 $OUT/tests_beta.log; exit 1; }
tail -3 $OUT/tests_beta.log
S="--set k_b1024:node_budget=1024"
S="$S --set pg0_b1024:branch=pgap,lookahead=0,node_budget=1024"
S="$S --set pg8_b1024:branch=pgap,lookahead=8,node_budget=1024"
S="$S --set pg0_b4096:branch=pgap,lookahead=0,node_budget=4096"
S="$S --set pg8_b4096:branch=pgap,lookahead=8,node_budget=4096"
timeout -k 10 600 python -u tools/exp/beta_residue.py --npz profiles/r6/res/relaxedBM_BM-8_unknown.npz --n 200 $S > $OUT/res_bm8.log 2>&1 || { tail -30 $OUT/res_bm8.log; exit 1; }
cat $OUT/res_bm8.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --budget-pass 0 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
