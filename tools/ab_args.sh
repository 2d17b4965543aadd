#!/bin/bash
# Alternating A/B of bench.py argument sets on ONE lease (verdict r2 item 7: >= 3 alternating runs
# per arm, median and spread):
#   bash tools/ab_args.sh OUT REPS "NAME1=ARGS1" "NAME2=ARGS2" ...      ("_" separates arguments)
# An arm "NAME=E/VAR=VAL/ARGS" also sets one environment variable (FAIRIFY_* A/B switches).
# Each run: bench.py --steps 3 --warmup 1 --budget-pass 0 plus the arm's arguments; JSON to
# OUT/<name>.<rep>.json; tools/ab_summary.py OUT prints the per-arm median / min / max table.
set -o pipefail
OUT=gpurun_out/$1; shift
REPS=$1; shift
mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for arm in "$@"; do
    name=${arm%%=*}; a=${arm#*=}
    ev=""
    if [ "${a:0:2}" = "E/" ]; then      # "E/VAR=VAL/ARGS": one environment variable for this arm
      rest=${a:2}; ev=${rest%%/*}; a=${rest#*/}; [ "$a" = "$rest" ] && a=""
    fi
    env $ev timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --budget-pass 0 ${a//_/ } > $OUT/$name.$rep.json 2> $OUT/$name.$rep.err || exit 1
    python -c "import json;d=json.load(open('$OUT/$name.$rep.json'));print('$name', $rep, d['ms_per_step'], d['pct_verified'], d['pct_verified_sound'])"
  done
done
python tools/ab_summary.py $OUT
