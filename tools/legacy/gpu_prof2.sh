#!/bin/bash
# Per-model diag + kernel stats of the default bench + PMC of the bound kernel (AC-4, AC-1).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/prof gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 600 python tools/diag_models.py --json-out gpurun_out/diag_models.json > gpurun_out/diag.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 1 --warmup 0 > gpurun_out/prof/bench_stdout.txt 2>&1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d gpurun_out/pmc/p1 -o run -- python3 tools/bench_bounds.py --models AC-4,AC-1 --iters 3 > gpurun_out/pmc/p1.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d gpurun_out/pmc/p2 -o run -- python3 tools/bench_bounds.py --models AC-4,AC-1 --iters 3 > gpurun_out/pmc/p2.txt 2>&1
echo done
