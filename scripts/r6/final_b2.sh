#!/bin/bash
# round 6 final one-HEAD baseline, call 2: targeted2, Table V, relaxed/GC, relaxed/BM, relaxed/AC without AC-7
set -o pipefail
export BASE_OUT=gpurun_out/r6fin
TLIM=250 bash scripts/r6/base.sh targeted2/BM && TLIM=60 bash scripts/r6/base.sh targeted2/GC && TLIM=200 bash scripts/r6/base.sh tablev && \
TLIM=60 bash scripts/r6/base.sh relaxed/GC && TLIM=250 bash scripts/r6/base.sh relaxed/BM && \
TLIM=250 bash scripts/r6/base.sh relaxed/AC AC-1,AC-2,AC-3,AC-4,AC-5,AC-6 && \
TLIM=150 bash scripts/r6/base.sh relaxed/AC AC-8,AC-9,AC-10,AC-11,AC-12
