#!/bin/bash
# Round 6: bn_stats_fused slice count A/B (16-byte phase-1 loads) on the BN per-launch table.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6bnsl; mkdir -p $o
for v in 32 64 128; do
  UNET_BN_SLICES=$v UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 \
    --norm batch --out $o/lt_bn_$v.md > $o/lt_bn_$v.log 2>&1 || { echo "lt bn rc=$?"; tail -20 $o/lt_bn_$v.log; exit 1; }
  head -3 $o/lt_bn_$v.md | tail -1
  grep -E "^\| bnfin" $o/lt_bn_$v.md
  grep -E "bnfin" $o/lt_bn_$v.md | head -20 | awk -F'|' '{printf "%s %s;", $3, $4} END {print ""}'
done
