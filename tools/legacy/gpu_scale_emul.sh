#!/bin/bash
# Strong-scaling emulation on one GPU: one rank's shard of an N-rank job, auto vs fixed chunk;
# and the CLI runner with 1 vs 4 concurrent streams.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/scale
for spec in "0/8:0" "0/8:4096" "0/4:0" "0/2:0"; do
  sh=${spec%%:*}; ch=${spec##*:}; tag=$(echo $sh | tr / _)_c$ch
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --emulate-shard $sh --chunk $ch --json-out gpurun_out/scale/$tag.json > gpurun_out/scale/$tag.log 2>&1
  python -c "import json; d=json.load(open('gpurun_out/scale/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['pct_verified'], d['config']['chunk'])"
done
for c in 1 4; do
  timeout -k 10 300 python -m fairify_amd.cli verify --preset src/AC-sex --weights random --models AC-4,AC-7 --out gpurun_out/scale/cli_c$c --no-accuracy --concurrency $c > gpurun_out/scale/cli_c$c.log 2>&1
  grep "partitions/s" gpurun_out/scale/cli_c$c.log | head -2
done
