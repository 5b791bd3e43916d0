#!/bin/bash
# Round 5 check G: the fp32 step test (float64 oracle), the wide-row kernels (first layer
# on 256 / 512-wide rows, tconv forward and composite wgrad on 128-wide coarse rows) and
# their effect on the 512^2 config; ATen fp32 upsampling step with MIOpen's NORMAL find
# mode (FAST picked naive fp32 NHWC kernels: 3.6 s per step in run E).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5g; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_tconv_fused.py \
  "tests/test_gpu_kernels.py::test_conv_first_layer_smallc" "tests/test_gpu_kernels.py::test_tconv_fwd_shuffle_and_dgrad" \
  -q -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed|vs float64" $o/tests.log | tail -8
[ $rc -gt 1 ] && { echo "tests crashed rc=$rc"; tail -30 $o/tests.log; exit 1; }
[ $rc -eq 1 ] && grep -E "^FAILED|Error" $o/tests.log | head -20
timeout -k 10 300 python bench.py --img_size 512 --in_channels 1 --per_gpu_batch 32 --steps 8 --warmup 3 > $o/s512.log 2>&1 \
  || { echo "s512 rc=$?"; tail -20 $o/s512.log; exit 1; }
grep '^{' $o/s512.log | cut -c1-160
timeout -k 10 300 python tools/layer_times.py --batch 32 --img 512 --in_channels 1 --reps 5 \
  --out $o/layer_times_s512_b32.md > $o/lt512.log 2>&1 || { echo "lt512 rc=$?"; tail -20 $o/lt512.log; exit 1; }
head -3 $o/layer_times_s512_b32.md | tail -1
grep -E "transConv8|conv1a" $o/layer_times_s512_b32.md | head -8
export MIOPEN_FIND_MODE=NORMAL
s=$(date +%s)
timeout -k 10 400 python train.py --synthetic --use_upsampling --in_channels 1 --img_size 128 --batch_size 256 \
  --synthetic_train 2560 --synthetic_test 256 --steps 12 --log_every 1 --no_checkpoint --noexport --noprogress \
  --backend torch --dtype fp32 --log_jsonl $o/aten_normal.jsonl > $o/aten_normal.log 2>&1 \
  || { echo "aten normal rc=$?"; tail -20 $o/aten_normal.log; exit 1; }
echo "ATen fp32 ups, MIOPEN_FIND_MODE=NORMAL: 12 steps in $(( $(date +%s) - s )) s"
python - $o/aten_normal.jsonl <<'PY'
import json, sys
r = [json.loads(l) for l in open(sys.argv[1])]
print([round(x["images_per_sec"], 1) for x in r if x["kind"] == "train"])
PY
