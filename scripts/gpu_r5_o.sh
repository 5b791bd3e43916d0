#!/bin/bash
# Round 5 check O: tconv data gradient on 128/256-wide coarse rows; 512^2 b32 bench + times.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5o; mkdir -p $o
timeout -k 10 600 python -u -m pytest "tests/test_gpu_kernels.py::test_tconv_fwd_shuffle_and_dgrad" \
  tests/test_gpu_tconv_fused.py -q -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed" $o/tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $o/tests.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --img_size 512 --in_channels 1 --per_gpu_batch 32 --steps 8 --warmup 3 > $o/s512.log 2>&1 \
  || { echo "s512 rc=$?"; tail -20 $o/s512.log; exit 1; }
grep '^{' $o/s512.log | cut -c1-160
timeout -k 10 300 python tools/layer_times.py --batch 32 --img 512 --in_channels 1 --reps 5 \
  --out $o/layer_times_s512_b32.md > $o/lt512.log 2>&1 || { echo "lt512 rc=$?"; tail -20 $o/lt512.log; exit 1; }
head -3 $o/layer_times_s512_b32.md | tail -1
grep -E "transConv9" $o/layer_times_s512_b32.md | head -6
