#!/bin/bash
# Full stress grids on one MI355X with the CLI runner (reference's trained weights):
# stress/AC = 3 290 112 partitions per model, stress/BM = 1 002 000.  CSVs stay on the box
# (hundreds of MB); summaries come back.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/stress
OUT=/tmp/stress_out
for spec in "stress/AC:AC-9" "stress/AC:AC-1" "stress/AC:AC-3" "stress/BM:BM-6" "stress/BM:BM-1"; do
  pre=${spec%%:*}; m=${spec##*:}; tag=$(echo $pre | tr / _)_$m
  timeout -k 10 ${PER_MODEL_TIMEOUT:-290} python -m fairify_amd.cli verify --preset $pre --models $m --out $OUT/$tag \
    --hard-timeout ${HARD:-240} > gpurun_out/stress/$tag.log 2>&1
  tail -3 gpurun_out/stress/$tag.log
  cp $OUT/$tag/summary.json gpurun_out/stress/$tag.summary.json
  ls -la $OUT/$tag/*.csv | tail -1
done
