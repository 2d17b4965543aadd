#!/bin/bash
# Table V with the reference's trained weights, anytime mode (growing BaB budgets + falsifier + MILP
# rounds on the residue within BUDGET seconds per model):  bash tools/gpu_tablev_anytime.sh OUT BUDGET PRESET...
set -o pipefail
OUT=$1; BUDGET=$2; shift 2
for P in "$@"; do
  tag=${P//\//_}
  bash tools/gpu_anytime.sh $OUT/$tag $P $(python -c "from fairify_amd import presets; print(','.join(presets.get('$P').models))") $BUDGET || exit $?
done
