#!/bin/bash
# First GPU validation: kernel tests, smoke, short bench.  Each GPU step has its own timeout.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -c "import torch; print(torch.cuda.get_device_name(0), torch.version.hip)"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke
timeout -k 10 600 python bench.py --scope chunk --chunk 2048 --models AC-1,AC-3,AC-9 --steps 1 --warmup 1 --json-out gpurun_out/bench_small.json
