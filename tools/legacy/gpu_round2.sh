#!/bin/bash
# After the backward bounds: GPU tests, smoke, default bench, scaling shards, Table V (trained
# weights) through the CLI, and a rocprofv3 kernel-stats pass of the default bench.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --json-out $O/bench.json > $O/bench.log 2>&1
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['ms_per_step'], d['value'], d['pct_verified'])"
for sh in 0/2 0/4 0/8 7/8; do
  tag=$(echo $sh | tr / _)
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --emulate-shard $sh --json-out $O/shard_$tag.json > $O/shard_$tag.log 2>&1
  python -c "import json; d=json.load(open('$O/shard_$tag.json')); print('$sh', d['ms_per_step'], d['value'], d['pct_verified'])"
done
for pre in src/AC-sex src/AC-race src/BM-age src/GC-age src/GC-sex; do
  tag=$(echo $pre | tr / _)
  timeout -k 10 300 python -u -m fairify_amd.cli verify --preset $pre --out /tmp/tv_$tag > $O/tv_$tag.log 2>&1
  cp /tmp/tv_$tag/summary.json $O/tv_$tag.summary.json
  grep -v "round " $O/tv_$tag.log | grep "\] " | wc -l
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 1 --warmup 1 --concurrency 4 > $O/prof_bench.log 2>&1
python tools/trace_busy.py $O/prof/run_kernel_trace.csv || true
rm -f $O/prof/run_kernel_trace.csv
