#!/bin/bash
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/crown2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_symbolic_kernel_gpu.py tests/test_bab_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --json-out $O/bench.json > $O/bench.log 2>&1
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['ms_per_step'], d['value'], d['pct_verified'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 1 --warmup 1 --concurrency 4 > $O/prof_bench.log 2>&1
python tools/trace_busy.py $O/prof/run_kernel_trace.csv || true
rm -f $O/prof/run_kernel_trace.csv
