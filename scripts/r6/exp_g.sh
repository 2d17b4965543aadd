#!/bin/bash
# round 6, call G: profiles of the beta stage -- kernel trace + stats of the BM-8 residue run (native
# loop, pgap) and of a stress/AC AC-7 slice, two PMC passes of fa_beta_kernel
set -o pipefail
OUT=gpurun_out/r6g; mkdir -p $OUT
R=$(pwd)
RES="$R/tools/exp/beta_residue.py --npz $R/tools/exp/data/relaxedBM_BM-8_unknown.npz --n 200 --set pg8:node_budget=1024"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/tr_res -o run -- python3 $RES > $R/$OUT/tr_res.log 2>&1 || { tail -20 $R/$OUT/tr_res.log; exit 1; }
tail -2 $R/$OUT/tr_res.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/tr_ac7 -o run -- python3 $R/tools/baseline_configs.py --group stress/AC --models AC-7 --max-partitions 100000 --out $R/$OUT/ac7 > $R/$OUT/tr_ac7.log 2>&1 || { tail -20 $R/$OUT/tr_ac7.log; exit 1; }
tail -2 $R/$OUT/tr_ac7.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d $R/$OUT/pmc1 -o run -- python3 $RES > $R/$OUT/pmc1.log 2>&1 || { tail -20 $R/$OUT/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS --output-format csv -d $R/$OUT/pmc2 -o run -- python3 $RES > $R/$OUT/pmc2.log 2>&1 || { tail -20 $R/$OUT/pmc2.log; exit 1; }
cd $R
for t in $(find $OUT/tr_res $OUT/tr_ac7 -name '*kernel_trace.csv'); do
  python tools/trace_busy.py $t > $t.busy.txt || true
  rm -f $t
done
python tools/pmc_summary.py $(find $OUT/pmc1 $OUT/pmc2 -name '*counter_collection.csv') > $OUT/pmc_beta.md
find $OUT/pmc1 $OUT/pmc2 -name '*counter_collection.csv' -delete
head -30 $OUT/pmc_beta.md
