#!/bin/bash
# TM=10 register-resident symbolic kernel (BM-4's 150-wide layer): numerics tests, micro-bench A/B
# against the LDS-tiled kernel, src/BM BM-4 verify; then a second escalation-filter sweep.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/tm10
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_symbolic_kernel_gpu.py tests/test_bab_gpu.py > gpurun_out/tm10/pytest.log 2>&1
tail -2 gpurun_out/tm10/pytest.log
for tm in 10 7; do
  FAIRIFY_SYM_MAX_TM=$tm timeout -k 10 120 python tools/bench_bounds.py --preset src/BM-age --models BM-4,BM-1 --rows 65536 --json-out gpurun_out/tm10/bb_tm$tm.json > gpurun_out/tm10/bb_tm$tm.log 2>&1
  echo "max_tm=$tm"; grep -i "BM-" gpurun_out/tm10/bb_tm$tm.log | head -4
done
timeout -k 10 200 python -m fairify_amd.cli verify --preset stress/BM --models BM-4 --out /tmp/bm4 --max-partitions 200000 --no-accuracy > gpurun_out/tm10/bm4.log 2>&1
grep "BM-4:" gpurun_out/tm10/bm4.log | tail -1
for spec in 16384:1024 8192:768 32768:768; do
  e=${spec%%:*}; o=${spec##*:}
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --escalate-budget $e --escalate-max-open $o \
    --json-out gpurun_out/tm10/e${e}_o${o}.json > gpurun_out/tm10/e${e}_o${o}.log 2>&1
  python -c "import json; d=json.load(open('gpurun_out/tm10/e${e}_o${o}.json')); print('e=$e o=$o', d['ms_per_step'], d['value'], d['pct_verified'])"
done
