#!/bin/bash
# round 6, call Z: kernel trace + stats of the final default bench step (1 step, no budget pass)
set -o pipefail
OUT=gpurun_out/r6z; mkdir -p $OUT
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/tr -o run -- python3 $R/bench.py --steps 1 --warmup 1 --budget-pass 0 > $R/$OUT/bench.json 2> $R/$OUT/bench.err || { tail -20 $R/$OUT/bench.err; exit 1; }
cd $R
for t in $(find $OUT/tr -name '*kernel_trace.csv'); do
  python tools/trace_busy.py $t > $OUT/trace_busy.txt || true
  rm -f $t
done
head -16 $OUT/trace_busy.txt
