#!/bin/bash
# BatchNorm step counters: wave-cycle stall pass + the PMC table passes (MFMA / VALU /
# LDS, FETCH_SIZE, WRITE_SIZE), each pass a run of its own
set -o pipefail
export TMPDIR=/tmp
bash scripts/gpu_stall_pmc.sh bn --norm batch || exit 1
python tools/stall_table.py $(find gpurun_out/stall_bn/pmc1 -name "*.db" | head -1) > gpurun_out/stall_bn/stall_table.md || exit 1
o=gpurun_out/prof_bn; rm -rf $o; mkdir -p $o
pass=0
for ctr in "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  pass=$((pass+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctr -d $o/pmc$pass -o run -- \
    python bench.py --steps 2 --warmup 1 --hip_graph 0 --norm batch > $o/pmc$pass.log 2>&1 || exit $?
done
python tools/pmc_table.py $o > $o/pmc_table.md
head -30 gpurun_out/stall_bn/stall_table.md
