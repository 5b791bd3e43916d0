#!/bin/bash
# Round 6 evidence: rocprofv3 kernel stats of the headline / BN / GN fp16 steps, per-launch
# tables of GN fp16, 512^2 b32 and 3D b8.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6prof; mkdir -p $o
( while sleep 50; do date >> $o/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
for cfg in "head:" "bn:--norm batch" "gn16:--norm group --dtype fp16"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  rm -rf $o/ks_$tag
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_$tag -o run -- \
    python bench.py --steps 5 --warmup 2 --hip_graph 0 $args > $o/ks_$tag.log 2>&1 || { echo "ks $tag rc=$?"; tail $o/ks_$tag.log; exit 1; }
  f=$(find $o/ks_$tag -name "*kernel_stats.csv" | head -1); cp $f $o/kstats_$tag.csv
done
UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --norm group --dtype fp16 \
  --out $o/lt_gn16.md > $o/lt_gn16.log 2>&1 || { echo "lt gn rc=$?"; tail -20 $o/lt_gn16.log; exit 1; }
UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 32 --img 512 --in_channels 1 \
  --out $o/lt_s512_b32.md > $o/lt_s512.log 2>&1 || { echo "lt 512 rc=$?"; tail -20 $o/lt_s512.log; exit 1; }
UNET_ENGINE="fwd_streams=1" timeout -k 10 400 python tools/layer_times.py --batch 8 --img 128 --dims 3 \
  --out $o/lt_3d_b8.md > $o/lt_3d.log 2>&1 || { echo "lt 3d rc=$?"; tail -20 $o/lt_3d.log; exit 1; }
head -3 $o/lt_gn16.md $o/lt_s512_b32.md $o/lt_3d_b8.md
