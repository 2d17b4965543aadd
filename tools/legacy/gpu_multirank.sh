#!/bin/bash
# Rehearsal of the multi-rank bench path on ONE GPU: 2 ranks share the device, host (gloo)
# collectives; checks torchrun launch, barriers, MAX/SUM reductions and the JSON line.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 FAIRIFY_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --concurrency 4 --json-out gpurun_out/bench_2rank_1gpu.json
cat gpurun_out/bench_2rank_1gpu.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29534 -m fairify_amd.cli verify --preset src/GC-age --weights zoo --out gpurun_out/mr_gc --no-accuracy
