#!/bin/bash
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/fals
M=AC-4,AC-7,AC-8,AC-11,AC-1
timeout -k 10 300 python tools/diag_models.py --models $M --residual-samples 0 > gpurun_out/fals/none.log 2>&1
timeout -k 10 300 python tools/diag_models.py --models $M --residual-samples 8192 --residual-iters 0 > gpurun_out/fals/samp.log 2>&1
timeout -k 10 300 python tools/diag_models.py --models $M --residual-samples 32768 --residual-iters 0 > gpurun_out/fals/samp32k.log 2>&1
timeout -k 10 300 python tools/diag_models.py --models $M --residual-samples 8192 --residual-iters 12 > gpurun_out/fals/ls12.log 2>&1
timeout -k 10 300 python tools/diag_models.py --models $M --residual-samples 8192 --residual-iters 12 --node-budget 8192 > gpurun_out/fals/ls12_b8k.log 2>&1
echo done
