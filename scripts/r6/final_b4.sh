#!/bin/bash
# round 6 final one-HEAD baseline, call 4: relaxed/AC AC-7 second half; then the GPU test tier and the bench
set -o pipefail
export BASE_OUT=gpurun_out/r6fin
TLIM=1000 bash scripts/r6/base.sh relaxed/AC AC-7 1645056
