set -o pipefail
mkdir -p gpurun_out/symb
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/symb/pmc1 -o run -- python3 $R/tools/bench_bounds.py --models AC-1,AC-12,AC-4 --rows 131072 --iters 2 > $R/gpurun_out/symb/pmc1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/symb/pmc2 -o run -- python3 $R/tools/bench_bounds.py --models AC-1,AC-12,AC-4 --rows 131072 --iters 2 > $R/gpurun_out/symb/pmc2.log 2>&1
