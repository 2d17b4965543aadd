#!/bin/bash
# Tests + micro-bench + PMC counters of the symbolic bound kernel (AC-4 and AC-1 shapes).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_symbolic_kernel_gpu.py tests/test_kernels_gpu.py tests/test_bab_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_symk.log 2>&1 || { tail -80 gpurun_out/pytest_symk.log; exit 1; }
tail -2 gpurun_out/pytest_symk.log
timeout -k 10 300 python tools/bench_bounds.py --json-out gpurun_out/bb_new.json
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
WANT="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F32 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
HAVE=""
for c in $WANT; do if grep -qw "$c" gpurun_out/pmc/counters.txt; then HAVE="$HAVE $c"; fi; done
echo "counters available: $HAVE"
set -- $HAVE
P1="$1 $2 $3 $4 $5 $6 $7 $8"; shift 8 || true
P2="$*"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d gpurun_out/pmc/p1 -o run -- python3 tools/bench_bounds.py --models AC-4,AC-1 --iters 3 > gpurun_out/pmc/p1.txt 2>&1
if [ -n "$P2" ]; then timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d gpurun_out/pmc/p2 -o run -- python3 tools/bench_bounds.py --models AC-4,AC-1 --iters 3 > gpurun_out/pmc/p2.txt 2>&1; fi
ls -R gpurun_out/pmc | head -30
