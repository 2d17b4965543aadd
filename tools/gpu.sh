#!/bin/bash
# One parameterised launcher for GPU-box work (run through gpurun from the repo root):
#
#   bash tools/gpu.sh OUT STEP [STEP ...]
#
# OUT is a directory under gpurun_out/; each STEP is one of
#   tests[:PYTEST_K]          GPU test tier (optionally -k filter)
#   bench[:ARGS]              bench.py with ARGS ("_" separates arguments), JSON to OUT/bench*.json
#   envbench:VAR=VAL[:ARGS]   the same with one environment variable set (A/B of FAIRIFY_* switches)
#   profpy:SCRIPT[:ARGS]      rocprofv3 --kernel-trace --stats of python SCRIPT ARGS (trace reduced to
#                             OUT/profN.busy.txt, then deleted)
#   prof[:ARGS]               rocprofv3 --kernel-trace --stats of bench.py ARGS (the trace csv is
#                             reduced to OUT/profN.busy.txt (whole run) and OUT/profN.window.txt (timed
#                             steps only, between bench.py's marker kernels) by tools/trace_busy.py, then deleted;
#                             the stats csv kept), default host concurrency
#   pmc:COUNTERS[:ARGS]       one rocprofv3 --pmc pass (counters comma-separated)
#   py:SCRIPT[:ARGS]          python SCRIPT ARGS
# Every GPU step runs under its own time limit; the first failing step ends the script.
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export PYTHONFAULTHANDLER=1
ROOT=$(pwd)
n=0
for step in "$@"; do
  n=$((n+1))
  kind=${step%%:*}; rest=${step#*:}; [ "$rest" = "$step" ] && rest=""
  args=${rest//_/ }
  case $kind in
    tests)
      # -k expression: "_" separates words (tests:decode_or_bab -> -k "decode or bab")
      if [ -n "$rest" ]; then
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$args" > $OUT/tests$n.log 2>&1
      else
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests$n.log 2>&1
      fi
      rc=$?; tail -5 $OUT/tests$n.log ;;
    bench)
      timeout -k 10 600 python -u bench.py $args > $OUT/bench$n.json 2> $OUT/bench$n.err
      rc=$?; cat $OUT/bench$n.json; [ $rc -ne 0 ] && tail -20 $OUT/bench$n.err ;;
    envbench)
      ev=${rest%%:*}; a2=${rest#*:}; [ "$a2" = "$rest" ] && a2=""
      env "$ev" timeout -k 10 600 python -u bench.py ${a2//_/ } > $OUT/bench$n.json 2> $OUT/bench$n.err
      rc=$?; cat $OUT/bench$n.json; [ $rc -ne 0 ] && tail -20 $OUT/bench$n.err ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $ROOT/$OUT/prof$n -o run -- python3 -u $ROOT/bench.py $args > $ROOT/$OUT/prof$n.out 2> $ROOT/$OUT/prof$n.err)
      rc=$?
      for t in $(find $OUT/prof$n -name '*kernel_trace.csv'); do
        python tools/trace_busy.py $t > $OUT/prof$n.busy.txt
        python tools/trace_busy.py $t --window > $OUT/prof$n.window.txt || true
      done
      find $OUT/prof$n -name '*kernel_trace.csv' -delete
      cat $OUT/prof$n.out; [ $rc -ne 0 ] && tail -30 $OUT/prof$n.err ;;
    profpy)
      # rocprofv3 kernel trace of any python script: profpy:SCRIPT:ARGS
      scr=${rest%%:*}; a2=${rest#*:}; [ "$a2" = "$rest" ] && a2=""
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $ROOT/$OUT/prof$n -o run -- python3 -u $ROOT/$scr ${a2//_/ } > $ROOT/$OUT/prof$n.out 2> $ROOT/$OUT/prof$n.err)
      rc=$?
      for t in $(find $OUT/prof$n -name '*kernel_trace.csv'); do
        python tools/trace_busy.py $t > $OUT/prof$n.busy.txt
      done
      find $OUT/prof$n -name '*kernel_trace.csv' -delete
      tail -5 $OUT/prof$n.out; [ $rc -ne 0 ] && tail -30 $OUT/prof$n.err ;;
    pmc)
      ctr=${rest%%:*}; a2=${rest#*:}; [ "$a2" = "$rest" ] && a2=""
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc ${ctr//,/ } --output-format csv \
        -d $ROOT/$OUT/pmc$n -o run -- python3 -u $ROOT/bench.py ${a2//_/ } > $ROOT/$OUT/pmc$n.out 2> $ROOT/$OUT/pmc$n.err)
      rc=$?; tail -2 $OUT/pmc$n.out ;;
    py)
      scr=${rest%%:*}; a2=${rest#*:}; [ "$a2" = "$rest" ] && a2=""
      timeout -k 10 900 python -u $scr ${a2//_/ } > $OUT/py$n.log 2>&1
      rc=$?; tail -30 $OUT/py$n.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "[gpu.sh] step $n ($kind) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
