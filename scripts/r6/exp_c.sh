#!/bin/bash
# round 6, call C: beta GPU tests (native runtime), BM-8 residue: primal-gap weighting / iterations /
# native vs torch loop; then the AC-7 stage breakdown slices (exp_b.sh)
set -o pipefail
OUT=gpurun_out/r6c; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
timeout -k 10 600 python -u -m pytest tests/test_beta_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/tests_beta.log 2>&1 || { tail -40 $OUT/tests_beta.log; exit 1; }
tail -3 $OUT/tests_beta.log
B="branch=pgap,lookahead=8,node_budget=1024"
S="--set pg8_torch:$B,native=0"
S="$S --set pg8:$B"
S="$S --set pg8_w2:$B,pgap_weights=2"
S="$S --set pg8_w3:$B,pgap_weights=3"
S="$S --set pg8_it128:$B,iters=128,root_iters=400"
S="$S --set pg8_it256:$B,iters=256,root_iters=800"
S="$S --set pg16:branch=pgap,lookahead=16,node_budget=1024"
S="$S --set pg8_w2_b4096:branch=pgap,lookahead=8,node_budget=4096,pgap_weights=2"
timeout -k 10 600 python -u tools/exp/beta_residue.py --npz tools/exp/data/relaxedBM_BM-8_unknown.npz --n 200 $S > $OUT/res_bm8.log 2>&1 || { tail -30 $OUT/res_bm8.log; exit 1; }
cat $OUT/res_bm8.log
bash scripts/r6/exp_b.sh
