#!/bin/bash
# Table-V style runs with the anytime mode on trained (zoo) weights: bash tools/gpu_anytime.sh OUT PRESET MODELS BUDGET
set -o pipefail
OUT=gpurun_out/$1; PRESET=$2; MODELS=$3; BUDGET=$4; shift 4
mkdir -p $OUT
export FAIRIFY_VERBOSE_ANYTIME=1 PYTHONFAULTHANDLER=1
timeout -k 10 1000 python -u -m fairify_amd.cli verify --preset $PRESET --models $MODELS --weights zoo \
  --node-budget 512 --escalate-budget 8192 --escalate-max-open 384 --anytime --anytime-budget $BUDGET \
  --out $OUT/res "$@" > $OUT/verify.log 2>&1
rc=$?; tail -25 $OUT/verify.log; exit $rc
