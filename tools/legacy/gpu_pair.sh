#!/bin/bash
# Paired-row symbolic kernel (two box rows per wave for single-tile networks): tests, A/B bench.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/pair
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
run() {
  tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --json-out $O/$tag.json > $O/$tag.log 2>&1
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', '$*', d['ms_per_step'], d['value'], d['pct_verified'])"
}
run pair --steps 2
FAIRIFY_SYM_PAIR=0 run single --steps 2
run pair_b --steps 2
FAIRIFY_SYM_PAIR=0 run single_b --steps 2
timeout -k 10 300 python tools/bench_bounds.py --models AC-1,AC-8,AC-9,AC-11,AC-12 --json-out $O/bb_pair.json > $O/bb_pair.log 2>&1
FAIRIFY_SYM_PAIR=0 timeout -k 10 300 python tools/bench_bounds.py --models AC-1,AC-8,AC-9,AC-11,AC-12 --json-out $O/bb_single.json > $O/bb_single.log 2>&1
tail -6 $O/bb_pair.log
tail -6 $O/bb_single.log
