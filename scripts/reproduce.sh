#!/bin/bash
# Reproduce the reference's experiment families on this node (replaces reproduce.sh /
# fairify.sh / the per-family copied drivers).
#
#   scripts/reproduce.sh [NGPU] [WEIGHTS] [OUT]
#
# NGPU    GPUs of this node (one rank per GPU, RCCL over xGMI); default 1
# WEIGHTS zoo (shipped Keras weights, converted) | random (synthetic benchmark setting)
# OUT     output root; each preset writes <OUT>/<preset>/<model>.csv + summary.json (Table V rows)
set -eo pipefail
NGPU=${1:-1}
WEIGHTS=${2:-zoo}
OUT=${3:-results}
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -m fairify_amd.csrc.build > /dev/null
run() {
  local preset=$1; shift
  if [ "$NGPU" -gt 1 ]; then
    python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NGPU" --master-addr 127.0.0.1 \
      --master-port $((29500 + RANDOM % 1000)) -m fairify_amd.cli verify --preset "$preset" \
      --weights "$WEIGHTS" --out "$OUT/$preset" "$@"
  else
    python -m fairify_amd.cli verify --preset "$preset" --weights "$WEIGHTS" --out "$OUT/$preset" "$@"
  fi
}
# Table V of the paper (src/ presets: soft 100 s, hard 30 min, P = 10 / 100)
for p in src/AC-sex src/AC-race src/GC-sex src/GC-age src/BM-age; do run "$p"; done
# fork suites
for p in src/CP src/CP12 src/DF; do run "$p"; done
# relaxed / targeted / targeted2 / stress families (grids up to 3.29 M partitions)
for p in relaxed/AC relaxed/GC relaxed/BM targeted/AC targeted/GC targeted/BM \
         targeted2/AC targeted2/GC targeted2/BM stress/GC stress/BM stress/AC; do
  run "$p" --escalate 4
done
python tools/table_v.py "$OUT"
