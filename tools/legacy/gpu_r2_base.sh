#!/bin/bash
# round-2 baseline on one MI355X: GPU tests, default bench, then the profiled default-concurrency
# bench with Python's faulthandler on (the profiler segfault investigation; runs last)
set -o pipefail
O=gpurun_out/r2base; mkdir -p $O
export PYTHONFAULTHANDLER=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 -u $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/$O/prof.out 2> $GRAFT_REPO_ROOT/$O/prof.err
echo "prof rc=$?"
tail -40 $GRAFT_REPO_ROOT/$O/prof.err
