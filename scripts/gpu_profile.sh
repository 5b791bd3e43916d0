#!/bin/bash
# Profiles of the current 1-GPU headline bench: rocprofv3 kernel stats, per-launch
# layer times, and three PMC passes (SQ: MFMA busy / VALU / LDS; TCC: FETCH_SIZE;
# WRITE_SIZE) -- one counter block set per run, each under its own time limit.
#   bash scripts/gpu_profile.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-cur}
o=gpurun_out/prof_$tag
rm -rf $o; mkdir -p $o
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks -o run -- \
  python bench.py --steps 5 --warmup 2 > $o/ks.log 2>&1 || exit $?
f=$(find $o/ks -name "*kernel_stats.csv" | head -1); cp $f $o/prof_kernel_stats.csv
python tools/prof_summary.py $o 7 "bench.py 2D 128x128x4 b${BATCH:-1024} bf16 ($tag)" > $o/kernel_stats.md || exit $?
UNET_ENGINE=fwd_streams=1 timeout -k 10 300 python tools/layer_times.py --batch ${BATCH:-1024} --img 128 --out $o/layer_times.md > $o/lt.log 2>&1 || exit $?
pass=0
for ctr in "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE"; do
  pass=$((pass+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctr -d $o/pmc$pass -o run -- \
    python bench.py --steps 2 --warmup 1 --hip_graph 0 > $o/pmc$pass.log 2>&1 || exit $?
done
python tools/pmc_table.py $o > $o/pmc_table.md
cat $o/kernel_stats.md | head -40
