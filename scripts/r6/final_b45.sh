#!/bin/bash
# round 6 final: relaxed/AC AC-7 second half, then the GPU test tier, smoke and the bench
set -o pipefail
bash scripts/r6/final_b4.sh && bash scripts/r6/final_b5.sh
