#!/bin/bash
# round 6, call P: the beta stage on stress/AC AC-7 (first 100 000 partitions, GPU stages only):
# kernel trace + stats, and two PMC passes restricted to fa_beta_kernel (after the kernel tuning)
set -o pipefail
OUT=gpurun_out/r6p; mkdir -p $OUT
R=$(pwd)
CMD="$R/tools/baseline_configs.py --group stress/AC --models AC-7 --max-partitions 100000"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/tr -o run -- python3 $CMD --out $R/$OUT/tr_run > $R/$OUT/tr.log 2>&1 || { tail -20 $R/$OUT/tr.log; exit 1; }
grep "AC-7" $R/$OUT/tr.log | tail -1
timeout -s KILL 300 rocprofv3 --kernel-include-regex fa_beta_kernel --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d $R/$OUT/pmc1 -o run -- python3 $CMD --out $R/$OUT/p1_run > $R/$OUT/pmc1.log 2>&1 || { tail -20 $R/$OUT/pmc1.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex fa_beta_kernel --pmc SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS --output-format csv -d $R/$OUT/pmc2 -o run -- python3 $CMD --out $R/$OUT/p2_run > $R/$OUT/pmc2.log 2>&1 || { tail -20 $R/$OUT/pmc2.log; exit 1; }
cd $R
for t in $(find $OUT/tr -name '*kernel_trace.csv'); do
  python tools/trace_busy.py $t > $OUT/trace_busy.txt || true
  rm -f $t
done
python tools/pmc_summary.py $(find $OUT/pmc1 $OUT/pmc2 -name '*counter_collection.csv') > $OUT/pmc_beta_ac7.md
find $OUT/pmc1 $OUT/pmc2 -name '*counter_collection.csv' -delete
head -14 $OUT/trace_busy.txt
head -6 $OUT/pmc_beta_ac7.md | cut -c1-400
