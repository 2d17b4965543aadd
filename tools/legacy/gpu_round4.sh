#!/bin/bash
# Deterministic BaB budget rule: GPU tests, smoke, default bench (2 steps), 2-rank rehearsal and a
# rocprofv3 kernel-stats pass of the default bench.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --json-out $O/bench.json > $O/bench.log 2>&1
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['ms_per_step'], d['value'], d['pct_verified'])"
export FAIRIFY_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --concurrency 4 --json-out $O/bench_2rank_1gpu.json > $O/bench2.log 2>&1
python -c "import json; d=json.load(open('$O/bench_2rank_1gpu.json')); print('2rank', d['ms_per_step'], d['value'], d['pct_verified'])"
unset FAIRIFY_DIST_BACKEND
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 1 --warmup 1 > $O/prof_bench.log 2>&1
python tools/trace_busy.py $O/prof/run_kernel_trace.csv > $O/busy.txt || true
rm -f $O/prof/run_kernel_trace.csv
cat $O/busy.txt | head -20
