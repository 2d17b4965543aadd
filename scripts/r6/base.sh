#!/bin/bash
# round 6 one-HEAD BASELINE configs: bash scripts/r6/base.sh GROUP [MODELS] [START] [N]
# (tools/baseline_configs.py; GPU stages only for the big grids, Table V in anytime mode); one call
# per part that fits the call limit, all parts under gpurun_out/r6base/ (report merges parts)
set -o pipefail
OUT=${BASE_OUT:-gpurun_out/r6base}; mkdir -p $OUT
G=$1; M=${2:-}; S=${3:-0}; N=${4:-}
HEAD=$(cat HEAD_SHA 2>/dev/null || echo "")
args="--group $G --out $OUT --head $HEAD"
[ -n "$M" ] && args="$args --models $M"
[ "$S" != "0" ] && args="$args --start $S"
[ -n "$N" ] && args="$args --max-partitions $N"
tag=$(echo "$G-$M-$S" | tr '/,' '__')
timeout -k 10 ${TLIM:-1140} python -u tools/baseline_configs.py $args > $OUT/$tag.log 2>&1
rc=$?
grep -v "^\[hb\]" $OUT/$tag.log | tail -14
exit $rc
