#!/bin/bash
# Host-side (Python) profile of the bench: cProfile, one thread (GIL contention removed).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/pyprof
timeout -k 10 600 python -m cProfile -o gpurun_out/pyprof/bench.pstats bench.py --concurrency 1 --steps 1 --warmup 1 > gpurun_out/pyprof/out.txt 2>&1
python - <<'PY'
import pstats
p = pstats.Stats("gpurun_out/pyprof/bench.pstats")
p.sort_stats("tottime").print_stats(35)
PY
