#!/bin/bash
# Round 6: fp32 executor kernel stats (b256), BN norm-head pass check.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6f32p; mkdir -p $o
( while sleep 50; do date >> $o/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
rm -rf $o/ks_f32
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/ks_f32 -o run -- \
  python bench.py --dtype fp32 --per_gpu_batch 256 --steps 4 --warmup 2 --hip_graph 0 > $o/ks_f32.log 2>&1 || { echo "ks rc=$?"; tail $o/ks_f32.log; exit 1; }
f=$(find $o/ks_f32 -name "*kernel_stats.csv" | head -1); cp $f $o/kstats_f32.csv
UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --norm batch \
  --out $o/lt_bn.md > $o/lt_bn.log 2>&1 || { echo "lt bn rc=$?"; tail -20 $o/lt_bn.log; exit 1; }
head -3 $o/lt_bn.md | tail -1
grep -E "fwd:Mask|bnfin:conv3a" $o/lt_bn.md
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py -k "norm_head or batch" > $o/t.log 2>&1 || { echo "t rc=$?"; tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
