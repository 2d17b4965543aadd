#!/bin/bash
# Every experiment preset end-to-end on one MI355X (first N partitions of the seeded order,
# shipped zoo weights where they exist): the reference's src/stress/relaxed/targeted/targeted2
# families and the fork's experiment drivers.  Writes gpurun_out/presets/<preset>/summary.json.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
N=${N:-512}
OUT=gpurun_out/presets
mkdir -p $OUT
for p in $(python -c "from fairify_amd import presets; print(' '.join(sorted(presets.PRESETS)))"); do
  timeout -k 10 300 python -m fairify_amd.cli verify --preset "$p" --weights zoo --out "$OUT/$p" \
    --max-partitions $N --no-accuracy --hard-timeout 120 > "$OUT/$(echo $p | tr / _).log" 2>&1 \
    || { echo "FAILED $p"; tail -20 "$OUT/$(echo $p | tr / _).log"; exit 1; }
  grep -h "partitions/s" "$OUT/$(echo $p | tr / _).log" | sed "s#^#$p #" | tail -20
done
python tools/table_v.py $OUT > $OUT/table_v.md
echo ok
