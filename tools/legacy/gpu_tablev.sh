#!/bin/bash
# Table V of the paper re-run on one MI355X with the reference's shipped (trained) weights:
# the src/ presets (soft 100 s / hard 30 min budgets, P = 10 / 100), full grids.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/tablev
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_determinism_gpu.py -x -q -p no:cacheprovider 2>&1 | tail -2
for p in src/GC-sex src/GC-age src/BM-age src/AC-sex src/AC-race; do
  timeout -k 10 900 python -m fairify_amd.cli verify --preset "$p" --weights zoo --out "$OUT/$p" --no-accuracy \
    > "$OUT/$(echo $p | tr / _).log" 2>&1 || { echo "FAILED $p"; tail -20 "$OUT/$(echo $p | tr / _).log"; exit 1; }
  grep -h "partitions/s" "$OUT/$(echo $p | tr / _).log" | tail -12
  rm -f $OUT/$p/*.csv
done
python tools/table_v.py $OUT > $OUT/table_v.md
echo ok
