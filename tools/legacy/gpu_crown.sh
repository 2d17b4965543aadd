#!/bin/bash
# CROWN kernel: numerics + soundness tests, native BaB tests, bench with and without it.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/crown
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_symbolic_kernel_gpu.py tests/test_bab_gpu.py tests/test_kernels_gpu.py > gpurun_out/crown/pytest.log 2>&1 || { tail -30 gpurun_out/crown/pytest.log; exit 1; }
tail -2 gpurun_out/crown/pytest.log
timeout -k 10 300 python bench.py --json-out gpurun_out/crown/bench_crown.json > gpurun_out/crown/bench_crown.log 2>&1
python -c "import json; d=json.load(open('gpurun_out/crown/bench_crown.json')); print('crown', d['ms_per_step'], d['value'], d['pct_verified'])"
FAIRIFY_CROWN=0 timeout -k 10 300 python bench.py --json-out gpurun_out/crown/bench_nocrown.json > gpurun_out/crown/bench_nocrown.log 2>&1
python -c "import json; d=json.load(open('gpurun_out/crown/bench_nocrown.json')); print('nocrown', d['ms_per_step'], d['value'], d['pct_verified'])"
