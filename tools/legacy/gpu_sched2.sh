#!/bin/bash
# Schedule variants with the deterministic open-frontier count.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/sched2
mkdir -p $O
run() {
  tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --json-out $O/$tag.json > $O/$tag.log 2>&1
  python -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', '$*', d['ms_per_step'], d['value'], d['pct_verified'])"
}
run B --node-budget 512 --escalate-max-open 127
run B2 --node-budget 512 --escalate-max-open 255
run C --escalate-max-open 127 --stages 32768:32
run D --escalate-budget 4096 --escalate-max-open 127 --stages 16384:48
run E --node-budget 256 --escalate-max-open 127
