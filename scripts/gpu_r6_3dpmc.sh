#!/bin/bash
# 3D b8 step counters: bytes fetched per kernel (FETCH_SIZE) and the wave-cycle split.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6_3dpmc; rm -rf $o; mkdir -p $o
pass=0
for ctr in "FETCH_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"; do
  pass=$((pass+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $o/pmc$pass -o run -- \
    python bench.py --dims 3 --per_gpu_batch 8 --steps 2 --warmup 1 --hip_graph 0 > $o/pmc$pass.log 2>&1 || exit $?
  python tools/pmc_summary.py $(find $o/pmc$pass -name "*.db" | head -1) wgrad > $o/summary$pass.txt || exit 1
done
cat $o/summary*.txt
