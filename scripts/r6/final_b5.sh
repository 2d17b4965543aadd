#!/bin/bash
# round 6 final: GPU test tier, smoke, default bench (3 runs)
set -o pipefail
OUT=gpurun_out/r6fin; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
for i in 1 2 3; do
  args="--steps 3 --warmup 1 --budget-pass 0"; [ "$i" = "1" ] && args=""
  timeout -k 10 300 python -u bench.py $args > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail -20 $OUT/bench_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$i.json'));print(d['ms_per_step'], d['value'], d['pct_verified_sound'], d['unknown'])"
done
