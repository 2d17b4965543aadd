#!/bin/bash
# Bound/point kernels: correctness tests, default bench, node-budget sweep on the hard models.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_symbolic_kernel_gpu.py tests/test_kernels_gpu.py tests/test_bab_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_symk.log 2>&1 || { tail -80 gpurun_out/pytest_symk.log; exit 1; }
tail -2 gpurun_out/pytest_symk.log
timeout -k 10 900 python bench.py --json-out gpurun_out/bench_symk.json
for b in 8192 32768; do
  timeout -k 10 600 python tools/diag_models.py --models AC-4,AC-7,AC-8,AC-11,AC-5 --node-budget $b --json-out gpurun_out/diag_b$b.json > gpurun_out/diag_b$b.log 2>&1
done
echo sweep done
