#!/bin/bash
# PMC comparison of the tconv-on-load consumer forward (conv_win XF 5) against the
# materialised-u one: two counter passes x UNET_ENGINE tconv_onload=0 / 2, one stream.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/utpmc; rm -rf $o; mkdir -p $o
p1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES"
p2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES"
p3="FETCH_SIZE"
for v in 0 2; do
  n=0
  for ctr in "$p1" "$p2" "$p3"; do
    n=$((n+1))
    UNET_ENGINE=fwd_streams=1,tconv_onload=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $o/u${v}_p$n -o run -- \
      python bench.py --steps 2 --warmup 1 --hip_graph 0 > $o/u${v}_p$n.log 2>&1 || exit $?
    python tools/pmc_summary.py $(find $o/u${v}_p$n -name "*.db" | head -1) conv_win_kernel > $o/u${v}_p$n.txt || exit 1
    echo "done u$v p$n"
  done
done
