#!/bin/bash
# round 6, call B: where AC-7's time goes on the big grids (stage timers + per-stage node counts on
# slices of stress/AC and relaxed/AC), GPU stages only as in tools/baseline_configs.py
set -o pipefail
OUT=gpurun_out/r6c; mkdir -p $OUT
export PYTHONFAULTHANDLER=1
for spec in "stress/AC:200000" "relaxed/AC:50000"; do
  pre=${spec%%:*}; n=${spec#*:}
  timeout -k 10 500 python -u tools/baseline_configs.py --group $pre --models AC-7 --max-partitions $n \
    --out $OUT/slice > $OUT/slice_${pre//\//_}.log 2>&1 || { tail -30 $OUT/slice_${pre//\//_}.log; exit 1; }
  tail -3 $OUT/slice_${pre//\//_}.log
  python -c "
import json,sys; d=json.load(open('$OUT/slice/${pre//\//_}/summary.json'))
for r in d['models']: print(r['model'], r['SAT'], r['UNSAT'], r['UNK'], r['wall_s'], r.get('stage_nodes'), json.dumps(r.get('stage_s')))"
done
