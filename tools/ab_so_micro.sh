#!/bin/bash
# Alternating A/B of extension builds on a micro-benchmark script:
#   bash tools/ab_so_micro.sh OUT DIR SCRIPT REPS v1 v2 ...     ("_" in SCRIPT separates its args)
# Each DIR/_C.<v>.so is copied over the in-tree extension before `python SCRIPT ARGS`; output to
# OUT/<v>.<rep>.log.  The in-tree build of the last variant stays in place.
set -o pipefail
OUT=gpurun_out/$1; DIR=$2; SCRIPT=$3; REPS=$4; shift 4
mkdir -p $OUT
SO=$(ls fairify_amd/_C.cpython-*.so)
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    cp $DIR/_C.$v.so $SO || exit 1
    timeout -k 10 300 python -u ${SCRIPT//_/ } > $OUT/$v.$rep.log 2>&1 || { tail -20 $OUT/$v.$rep.log; exit 1; }
    echo "== $v rep $rep"; cat $OUT/$v.$rep.log
  done
done
