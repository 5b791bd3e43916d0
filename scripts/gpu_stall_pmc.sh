#!/bin/bash
# Wave-cycle breakdown (active / parked on waitcnt-barrier / issue-stalled) of the
# headline step's kernels: one SQ pass (8 counters), eager launches.
#   bash scripts/gpu_stall_pmc.sh <tag> [bench args]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-cur}; shift
o=gpurun_out/stall_$tag
rm -rf $o; mkdir -p $o
timeout -k 10 60 rocprofv3 -L > $o/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES -d $o/pmc1 -o run -- \
  python bench.py --steps 2 --warmup 1 --hip_graph 0 "$@" > $o/pmc1.log 2>&1 || exit $?
python tools/pmc_summary.py $(find $o/pmc1 -name "*.db" | head -1) > $o/summary.txt
