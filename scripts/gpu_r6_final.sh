#!/bin/bash
# Round 6 end: smoke, rocprofv3 kernel stats (headline / BN / GN fp16 / 3D), per-launch tables.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6final; mkdir -p $o
( while sleep 50; do date >> $o/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
for cfg in "head:" "bn:--norm batch" "gn16:--norm group --dtype fp16" "d3:--dims 3"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  rm -rf $o/ks_$tag
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_$tag -o prof -- \
    python bench.py --steps 5 --warmup 2 --hip_graph 0 $args > $o/ks_$tag.log 2>&1 || { echo "ks $tag rc=$?"; tail $o/ks_$tag.log; exit 1; }
  f=$(find $o/ks_$tag -name "*kernel_stats.csv" | head -1); mkdir -p $o/st_$tag; cp $f $o/st_$tag/prof_kernel_stats.csv
done
lt() { UNET_ENGINE="fwd_streams=1" timeout -k 10 400 python tools/layer_times.py ${@:2} --out $o/$1.md > $o/$1.log 2>&1 || { echo "lt $1 rc=$?"; tail -20 $o/$1.log; exit 1; }; head -3 $o/$1.md | tail -1; }
lt lt_head --batch 1024 --img 128
lt lt_bn --batch 1024 --img 128 --norm batch
lt lt_gn16 --batch 1024 --img 128 --norm group --dtype fp16
lt lt_3d --batch 8 --img 128 --dims 3
lt lt_s512 --batch 32 --img 512 --in_channels 1
