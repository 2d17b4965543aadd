#!/bin/bash
# Split-sample simulation kernel: numerics tests, then 1/8 shard and full bench A/B over FAIRIFY_SIM_BLOCKS.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/sim_split2
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "sim" -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
run() {
  tag=$1; shift
  timeout -k 10 200 python bench.py --json-out $O/$tag.json "$@" > $O/$tag.txt 2>&1 || { tail -20 $O/$tag.txt; return 1; }
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['ms_per_step'], round(d['value']), d['pct_verified'], d['sat'], d['unsat'], flush=True)"
}
run s08_off --steps 3 --warmup 1 --emulate-shard 0/8 &&
FAIRIFY_SIM_BLOCKS=512 run s08_b512 --steps 3 --warmup 1 --emulate-shard 0/8 &&
FAIRIFY_SIM_BLOCKS=1024 run s08_b1024 --steps 3 --warmup 1 --emulate-shard 0/8 &&
run s08_off2 --steps 3 --warmup 1 --emulate-shard 0/8 &&
FAIRIFY_SIM_BLOCKS=512 run full_b512 --steps 2 --warmup 1
