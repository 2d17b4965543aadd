#!/bin/bash
# Short GPU bench with stage profile. Usage: tools/gpu_bench.sh [extra bench args]
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python bench.py --profile "$@" 2> gpurun_out/bench_profile.txt | tee gpurun_out/bench.json
cat gpurun_out/bench_profile.txt | tail -30
