#!/bin/bash
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for v in "" "--bisect-steps 0" "--concurrency 12" "--chunk 8192"; do
  timeout -k 10 600 python bench.py $v --json-out gpurun_out/ab/x.json > /dev/null 2>&1
  python -c "import json;r=json.load(open('gpurun_out/ab/x.json'));print('$v', r['value'], r['ms_per_step'], r['pct_verified'])"
done
