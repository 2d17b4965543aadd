#!/bin/bash
# Certificate-kernel change: numerics tests + BaB tests + default bench + CLI verify with stream concurrency.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/cert
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_bab_gpu.py tests/test_determinism_gpu.py > gpurun_out/cert/pytest.log 2>&1
tail -2 gpurun_out/cert/pytest.log
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --json-out gpurun_out/cert/bench.json > gpurun_out/cert/bench.log 2>&1
tail -1 gpurun_out/cert/bench.log
timeout -k 10 300 python -m fairify_amd.cli verify --preset src/AC-sex --weights random --models AC-4,AC-8 --out gpurun_out/cert/ac --no-accuracy > gpurun_out/cert/verify.log 2>&1
tail -4 gpurun_out/cert/verify.log
