#!/bin/bash
# PMC counters of the bench's hot kernels (AC-4, AC-7, AC-1 of the default bench), one
# counter group per run (<= 8 SQ, <= 4 TCC), each pass under its own hard time limit.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/pmc2
mkdir -p $O
export TMPDIR=/tmp
CMD="python3 bench.py --models AC-4,AC-7,AC-1 --steps 1 --warmup 0 --concurrency 1"
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
pass() {
  tag=$1; shift
  HAVE=""
  for c in "$@"; do if grep -qw "$c" $O/counters.txt; then HAVE="$HAVE $c"; fi; done
  echo "$tag: $HAVE"
  [ -n "$HAVE" ] || return 0
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $HAVE --output-format csv -d $O/$tag -o run -- $CMD > $O/$tag.log 2>&1
}
pass p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES
pass p2 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
pass p3 FETCH_SIZE
pass p4 WRITE_SIZE
ls $O/*/ | head
python tools/pmc_summary.py $(ls $O/p*/run_counter_collection.csv) > $O/summary.md
head -40 $O/summary.md
rm -f $O/p*/run_kernel_trace.csv
