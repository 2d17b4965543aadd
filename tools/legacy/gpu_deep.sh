#!/bin/bash
# Per-model diagnostic with a deep-budget re-run of the UNKNOWN residue (how do they resolve?).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python tools/diag_models.py --json-out gpurun_out/diag_deep.json --residual-samples 2048 --residual-iters 12 "$@" > gpurun_out/diag_deep.log 2>&1 || { tail -40 gpurun_out/diag_deep.log; exit 1; }
cat gpurun_out/diag_deep.log
