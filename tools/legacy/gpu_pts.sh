#!/bin/bash
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python tools/bench_bounds.py --mode points --models AC-4,AC-5,AC-1
timeout -k 10 300 python tools/bench_bounds.py --mode points --models AC-4,AC-5,AC-1 --rows 4096
