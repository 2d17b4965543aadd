#!/bin/bash
# round 6, call AB: run-to-run identity of the AC-7 rows after the race fix (beta with the forward
# weights in LDS, WM 0): targeted/AC AC-7 twice, targeted2/AC AC-7 once (final rows: 3 520 / 15 113 UNKNOWN)
set -o pipefail
OUT=gpurun_out/r6ab; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 200 python -u tools/baseline_configs.py --group targeted/AC --models AC-7 --out $OUT/t_$i > $OUT/t_$i.log 2>&1 || { tail -30 $OUT/t_$i.log; exit 1; }
  grep "(zoo)" $OUT/t_$i.log
done
timeout -k 10 400 python -u tools/baseline_configs.py --group targeted2/AC --models AC-7 --out $OUT/t2 > $OUT/t2.log 2>&1 || { tail -30 $OUT/t2.log; exit 1; }
grep "(zoo)" $OUT/t2.log
