#!/bin/bash
# round 6, call Y (after the shaped kernels): all 8 emulated ranks of an 8-GPU bench step on one lease, next to N=1
set -o pipefail
OUT=gpurun_out/r6y; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --budget-pass 0 > $OUT/n1.json 2> $OUT/n1.err || { tail -20 $OUT/n1.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/n1.json'));print('N=1', d['ms_per_step'], d['pct_verified_sound'])"
bash tools/shard_ranks.sh r6y 8 FAIRIFY_NODE_W_C 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --budget-pass 0 > $OUT/n1b.json 2> $OUT/n1b.err || { tail -20 $OUT/n1b.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/n1b.json'));print('N=1 (after)', d['ms_per_step'], d['pct_verified_sound'])"
