#!/bin/bash
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/budget
for b in 2048 4096 8192; do
  timeout -k 10 600 python bench.py --node-budget $b --json-out gpurun_out/budget/b$b.json > /dev/null 2>&1
  cat gpurun_out/budget/b$b.json
done
timeout -k 10 600 python bench.py --node-budget 4096 --residual-samples 0 --json-out gpurun_out/budget/b4096_nofals.json > /dev/null 2>&1
cat gpurun_out/budget/b4096_nofals.json
