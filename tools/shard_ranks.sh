#!/bin/bash
# Every rank of an emulated N-rank job on this one GPU, for each setting of one environment
# variable (LPT cost-model A/B): bash tools/shard_ranks.sh OUT N VAR VAL1 VAL2 ...
# Each run: bench.py --emulate-shard r/N --steps 3 --warmup 1 --budget-pass 0; prints per-rank ms
# and, per value, the max / mean ratio (the straggler factor a real N-rank step pays).
set -o pipefail
OUT=gpurun_out/$1; N=$2; VAR=$3; shift 3
mkdir -p $OUT
for val in "$@"; do
  for r in $(seq 0 $((N - 1))); do
    env $VAR=$val timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --budget-pass 0 --emulate-shard $r/$N \
      > $OUT/$val.$r.json 2> $OUT/$val.$r.err || exit 1
  done
  python - "$OUT" "$val" "$N" <<'PY'
import json, sys
out, val, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
ms = [json.load(open(f"{out}/{val}.{r}.json"))["ms_per_step"] for r in range(n)]
print(val, "ranks ms", [round(m, 1) for m in ms], "max", round(max(ms), 1), "max/mean", round(max(ms) / (sum(ms) / n), 3))
PY
done
