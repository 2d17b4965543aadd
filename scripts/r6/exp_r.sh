#!/bin/bash
# round 6, call R: compile-time-shape symbolic and refine kernels (common.h FaShape) -- bitwise tests,
# per-model micro-benchmark, SALU:VALU PMC pass and the default bench, shaped vs run-time shape
# alternating on one lease; stress/AC AC-7 200 000-partition slice both ways
set -o pipefail
OUT=gpurun_out/r6r; mkdir -p $OUT
R=$(pwd)
export PYTHONFAULTHANDLER=1
timeout -k 10 400 python -u -m pytest tests/test_symbolic_kernel_gpu.py tests/test_refine_gpu.py tests/test_tightness_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do for s in 1 0; do
  FAIRIFY_SYM_SHAPED=$s FAIRIFY_REFINE_SHAPED=$s timeout -k 10 120 python tools/bench_bounds.py --models AC-2,AC-3,AC-4,AC-5,AC-7 --rows 131072 --iters 20 \
    --json-out $OUT/micro_s${s}_$i.json > $OUT/micro_s${s}_$i.log 2>&1 || { tail -20 $OUT/micro_s${s}_$i.log; exit 1; }
done; done
cd /tmp && export TMPDIR=/tmp
for s in 1 0; do
  FAIRIFY_SYM_SHAPED=$s FAIRIFY_REFINE_SHAPED=$s timeout -s KILL 200 rocprofv3 --kernel-include-regex 'fa_sym_kernel|fa_refine_kernel' --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/$OUT/pmc_s$s -o run -- python3 $R/bench.py --steps 1 --warmup 0 --budget-pass 0 > $R/$OUT/pmc_s$s.log 2>&1 || { tail -20 $R/$OUT/pmc_s$s.log; exit 1; }
done
cd $R
for s in 1 0; do
  python tools/pmc_summary.py $(find $OUT/pmc_s$s -name '*counter_collection.csv') > $OUT/pmc_sym_s$s.md
  find $OUT/pmc_s$s -name '*counter_collection.csv' -delete
  head -12 $OUT/pmc_sym_s$s.md | cut -c1-300
done
for i in 1 2 3; do for s in 1 0; do
  FAIRIFY_SYM_SHAPED=$s FAIRIFY_REFINE_SHAPED=$s timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --budget-pass 0 > $OUT/bench_s${s}_$i.json 2> $OUT/bench_s${s}_$i.err || { tail -20 $OUT/bench_s${s}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_s${s}_$i.json'));print('s$s', d['ms_per_step'], d['value'], d['pct_verified_sound'], d['unknown'])"
done; done
for s in 1 0; do
  FAIRIFY_SYM_SHAPED=$s FAIRIFY_REFINE_SHAPED=$s timeout -k 10 300 python -u tools/baseline_configs.py --group stress/AC --models AC-7 --max-partitions 200000 \
    --out $OUT/slice_s$s > $OUT/slice_s$s.log 2>&1 || { tail -30 $OUT/slice_s$s.log; exit 1; }
  grep "AC-7 (zoo)" $OUT/slice_s$s.log
done
