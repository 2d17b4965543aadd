#!/bin/bash
# Crown kernel with W^T staging + odd slab stride: tests, bench, LDS-conflict counters.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/crown3
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
run() {
  tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --json-out $O/$tag.json > $O/$tag.log 2>&1
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', '$*', d['ms_per_step'], d['value'], d['pct_verified'])"
}
run full --steps 2
run full_b --steps 2
export TMPDIR=/tmp
CMD="python3 bench.py --models AC-4,AC-7,AC-1 --steps 1 --warmup 0 --concurrency 1"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc -o run -- $CMD > $O/pmc.log 2>&1
python tools/pmc_summary.py $O/pmc/run_counter_collection.csv > $O/pmc_summary.md
rm -f $O/pmc/run_kernel_trace.csv
head -8 $O/pmc_summary.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 1 --warmup 1 > $O/prof_bench.log 2>&1
python tools/trace_busy.py $O/prof/run_kernel_trace.csv > $O/busy.txt || true
rm -f $O/prof/run_kernel_trace.csv
head -8 $O/busy.txt
