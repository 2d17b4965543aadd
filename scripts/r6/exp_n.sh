#!/bin/bash
# round 6, call N: cheap ways to decide more of the headline step's residue inside the timed step
# (alternating with the default on the same lease)
set -o pipefail
OUT=gpurun_out/r6n; mkdir -p $OUT
n=0
for spec in "def:" "mo768:--escalate-max-open_768" "rs8k:--residual-samples_8192" "def2:" "b64:--beta-budget_64" "mo768rs8k:--escalate-max-open_768_--residual-samples_8192"; do
  n=$((n+1)); tag=${spec%%:*}; a=${spec#*:}; a=${a//_/ }
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --budget-pass 0 $a > $OUT/$tag.json 2> $OUT/$tag.err || { tail -20 $OUT/$tag.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', d['ms_per_step'], d['value'], d['pct_verified_sound'], d['unknown'], {k: v['unknown'] for k, v in d['per_model'].items() if v['unknown']})"
done
