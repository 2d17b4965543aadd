#!/bin/bash
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 120 build/symk_timing 65536
timeout -k 10 120 build/symk_timing_noepi 65536
timeout -k 10 600 python -m pytest tests/test_symbolic_kernel_gpu.py tests/test_bab_gpu.py tests/test_determinism_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_symk.log 2>&1 || { tail -60 gpurun_out/pytest_symk.log; exit 1; }
tail -1 gpurun_out/pytest_symk.log
timeout -k 10 300 python tools/bench_bounds.py --json-out gpurun_out/bb_2tile.json
timeout -k 10 600 python bench.py --json-out gpurun_out/bench_2tile.json
