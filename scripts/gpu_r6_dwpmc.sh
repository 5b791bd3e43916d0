#!/bin/bash
# conv_dw counters (scripts/dw_micro.py launches): wave-cycle stalls, MFMA / VALU / LDS, bytes.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6dwpmc; rm -rf $o; mkdir -p $o
pass=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  pass=$((pass+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctr -d $o/pmc$pass -o run -- \
    python scripts/dw_micro.py 1024 2 > $o/pmc$pass.log 2>&1 || exit $?
  python tools/pmc_summary.py $(find $o/pmc$pass -name "*.db" | head -1) conv_dw > $o/summary$pass.txt || exit 1
done
cat $o/summary*.txt
