#!/bin/bash
# Full-grid runs of the relaxed / targeted presets (RA + tau semantics, domain overrides) on
# one MI355X with the CLI runner, reference weights; summaries come back, CSVs are deleted.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/presets_full
OUT=/tmp/presets_full
for spec in "relaxed/AC:AC-1,AC-3" "targeted/AC:AC-1,AC-3" "targeted2/AC:AC-1,AC-3" "relaxed/BM:BM-1,BM-6" "targeted/BM:BM-1,BM-6" "targeted2/BM:BM-1,BM-6" "relaxed/GC:GC-1,GC-3" "targeted/GC:GC-1,GC-3" "targeted2/GC:GC-1,GC-3" "stress/GC:GC-1,GC-3"; do
  pre=${spec%%:*}; models=${spec##*:}; tag=$(echo $pre | tr / _)
  timeout -k 10 ${TIMEOUT:-400} python -u -m fairify_amd.cli verify --preset $pre --models $models --out $OUT/$tag \
    --hard-timeout ${HARD:-150} --no-accuracy > gpurun_out/presets_full/$tag.log 2>&1
  grep -v "round " gpurun_out/presets_full/$tag.log | grep "\] " | tail -2
  cp $OUT/$tag/summary.json gpurun_out/presets_full/$tag.summary.json
  rm -rf $OUT/$tag
done
