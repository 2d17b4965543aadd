#!/bin/bash
# Round-end rehearsal (GPU tests, smoke, default bench, 2-rank path) + Table V re-run with the
# deterministic BaB (trained weights, CLI defaults).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --json-out $O/bench_default.json > $O/bench.log 2>&1
python -c "import json; d=json.load(open('$O/bench_default.json')); print('bench', d['ms_per_step'], d['value'], d['pct_verified'])"
export FAIRIFY_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --concurrency 4 --json-out $O/bench_2rank_1gpu.json > $O/bench2.log 2>&1
python -c "import json; d=json.load(open('$O/bench_2rank_1gpu.json')); print('2rank', d['ms_per_step'], d['value'], d['pct_verified'])"
unset FAIRIFY_DIST_BACKEND
for pre in src/AC-sex src/AC-race src/BM-age src/GC-age src/GC-sex; do
  tag=$(echo $pre | tr / _)
  timeout -k 10 300 python -u -m fairify_amd.cli verify --preset $pre --out /tmp/tv_$tag > $O/tv_$tag.log 2>&1
  cp /tmp/tv_$tag/summary.json $O/tv_$tag.summary.json
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5/tv_*.summary.json")):
    d = json.load(open(f))
    print(f, json.dumps(d)[:300])
PY
