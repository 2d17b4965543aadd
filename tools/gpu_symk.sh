#!/bin/bash
# Symbolic kernel: correctness tests, micro-bench, default bench.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_symbolic_kernel_gpu.py tests/test_kernels_gpu.py tests/test_bab_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_symk.log 2>&1 || { tail -80 gpurun_out/pytest_symk.log; exit 1; }
tail -2 gpurun_out/pytest_symk.log
timeout -k 10 300 python tools/bench_bounds.py --json-out gpurun_out/bb_new.json
timeout -k 10 900 python bench.py --json-out gpurun_out/bench_symk.json
