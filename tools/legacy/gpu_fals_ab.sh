#!/bin/bash
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/fab
for spec in "default|" "nofals|--residual-samples 0" "iters4|--residual-iters 4" "default2|"; do
  tag=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 $args --json-out gpurun_out/fab/$tag.json > gpurun_out/fab/$tag.log 2>&1
  python -c "import json; d=json.load(open('gpurun_out/fab/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['pct_verified'])"
done
