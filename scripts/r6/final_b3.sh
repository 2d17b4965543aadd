#!/bin/bash
# round 6 final one-HEAD baseline, call 3: relaxed/AC AC-7, first half of the seeded order
set -o pipefail
export BASE_OUT=gpurun_out/r6fin
TLIM=1100 bash scripts/r6/base.sh relaxed/AC AC-7 0 1645056
