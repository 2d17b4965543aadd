#!/bin/bash
# Round validation on one MI355X: GPU tests, smoke, default bench (whole AC suite), stage profile.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke
timeout -k 10 900 python bench.py --json-out gpurun_out/bench_default.json
timeout -k 10 900 python bench.py --steps 1 --warmup 1 --profile --json-out gpurun_out/bench_prof.json 2> gpurun_out/bench_profile.txt
tail -30 gpurun_out/bench_profile.txt
