#!/bin/bash
# Round 5 check H: first-layer window zero tail (W = 512 fix), GroupNorm two-stream forward
# (bit-identity tests + same-box A/B), 512^2 bench, ATen fp32 with MIOpen's NORMAL find mode
# (bench config and the upsampling-decoder Dice arm, seeds 1-3, 200 steps).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5h; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest "tests/test_gpu_kernels.py::test_conv_first_layer_smallc" \
  "tests/test_gpu_model.py::test_two_stream_forward_equals_one_stream" tests/test_gpu_norm_fused.py tests/test_gpu_f32.py \
  -q -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed" $o/tests.log | tail -4
[ $rc -gt 1 ] && { echo "tests crashed rc=$rc"; tail -30 $o/tests.log; exit 1; }
[ $rc -eq 1 ] && { grep -E "^FAILED|Error" $o/tests.log | head -20; exit 1; }
for r in 1 2; do
  for fs in 1 2; do
    UNET_ENGINE=fwd_streams=$fs timeout -k 10 300 python bench.py --norm group --dtype fp16 --steps 10 --warmup 3 \
      > $o/gn_fs${fs}_$r.log 2>&1 || { echo "gn fs$fs rc=$?"; tail -20 $o/gn_fs${fs}_$r.log; exit 1; }
    echo "GN fp16 fwd_streams=$fs run $r: $(grep '^{' $o/gn_fs${fs}_$r.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  done
done
timeout -k 10 300 python bench.py --img_size 512 --in_channels 1 --per_gpu_batch 32 --steps 8 --warmup 3 > $o/s512.log 2>&1 \
  || { echo "s512 rc=$?"; tail -20 $o/s512.log; exit 1; }
grep '^{' $o/s512.log | cut -c1-160
for cfg in "" "--use_upsampling --in_channels 1"; do
  timeout -k 10 300 python bench.py --dtype fp32 --per_gpu_batch 128 --steps 5 --warmup 2 $cfg > $o/f32.log 2>&1 \
    || { echo "native fp32 rc=$?"; tail -20 $o/f32.log; exit 1; }
  echo "native fp32 [$cfg]: $(grep '^{' $o/f32.log | cut -c1-120)"
  cp $o/f32.log "$o/f32_${cfg// /_}.log"
done
export MIOPEN_FIND_MODE=NORMAL
timeout -k 10 600 python bench.py --dtype fp32 --backend torch --per_gpu_batch 128 --steps 5 --warmup 2 > $o/aten32_normal.log 2>&1 \
  || { echo "aten fp32 normal rc=$?"; tail -20 $o/aten32_normal.log; exit 1; }
grep '^{' $o/aten32_normal.log | cut -c1-160
ARMS=aten_fp32 timeout -k 10 900 bash scripts/gpu_r5_ups_dice.sh 200 1 2 3 > $o/dice.log 2>&1 \
  || { echo "dice rc=$?"; tail -20 $o/dice.log; exit 1; }
grep -h "seed" $o/dice.log
