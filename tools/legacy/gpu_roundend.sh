#!/bin/bash
# Round-end rehearsal: what the driver runs (GPU tests, smoke, default bench) + 2-rank path.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/roundend
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/roundend/pytest_gpu.log 2>&1
tail -2 gpurun_out/roundend/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/roundend/smoke.log 2>&1
tail -1 gpurun_out/roundend/smoke.log
timeout -k 10 300 python bench.py --json-out gpurun_out/roundend/bench_default.json > gpurun_out/roundend/bench.log 2>&1
cat gpurun_out/roundend/bench_default.json
export FAIRIFY_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --concurrency 4 --json-out gpurun_out/roundend/bench_2rank_1gpu.json > gpurun_out/roundend/bench2.log 2>&1
cat gpurun_out/roundend/bench_2rank_1gpu.json
