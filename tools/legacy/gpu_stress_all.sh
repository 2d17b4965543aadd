#!/bin/bash
# Full stress grids on one MI355X through the CLI runner, reference (trained) weights:
# stress/AC = 3 290 112 partitions per model, stress/BM = 1 002 000.  MODELS_AC / MODELS_BM pick
# the models; CSVs (100s of MB) are sized then deleted; per-model summaries come back.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/stress_all
OUT=/tmp/stress_out
run() {
  local pre=$1 models=$2 tag=$(echo $1 | tr / _)_$3
  timeout -k 10 ${TIMEOUT:-900} python -u -m fairify_amd.cli verify --preset $pre --models $models --out $OUT/$tag \
    --hard-timeout ${HARD:-240} > gpurun_out/stress_all/$tag.log 2>&1
  grep -v "round " gpurun_out/stress_all/$tag.log | tail -12
  cp $OUT/$tag/summary.json gpurun_out/stress_all/$tag.summary.json
  du -sh $OUT/$tag
  rm -rf $OUT/$tag
}
[ -n "${MODELS_AC:-}" ] && run stress/AC $MODELS_AC b
[ -n "${MODELS_BM:-}" ] && run stress/BM $MODELS_BM a
if [ -n "${DIAG:-}" ]; then
  timeout -k 10 300 python tools/diag_escalate.py --json-out gpurun_out/stress_all/diag_escalate.json > gpurun_out/stress_all/diag_escalate.log 2>&1
  cat gpurun_out/stress_all/diag_escalate.log
fi
