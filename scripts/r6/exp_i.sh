#!/bin/bash
# round 6, call I: fa_beta_kernel occupancy A/B (register target FA_BETA_WPE 2 / 3 / 4, with the
# waves-per-CU launch config and the unrolled inner loops), alternating, on the BM-8 residue run
set -o pipefail
OUT=gpurun_out/r6i; mkdir -p $OUT
SO=$(ls fairify_amd/_C.cpython-*.so)
cp $SO $OUT/orig.so
for rep in 1 2; do
  for v in wpe2 wpe3 wpe4; do
    cp abvar6/_C.$v.so $SO || exit 1
    timeout -k 10 300 python -u tools/exp/beta_residue.py --npz tools/exp/data/relaxedBM_BM-8_unknown.npz --n 200 \
      --set $v:node_budget=1024 > $OUT/$v.$rep.log 2>&1 || { tail -20 $OUT/$v.$rep.log; exit 1; }
    tail -1 $OUT/$v.$rep.log
  done
done
cp $OUT/orig.so $SO
rm -f $OUT/orig.so
