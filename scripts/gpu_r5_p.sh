#!/bin/bash
# Round 5 check P: 3D first layer on the window kernel (tests, 3D model steps, 3D bench + times).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5p; mkdir -p $o
timeout -k 10 600 python -u -m pytest "tests/test_gpu_kernels.py::test_conv3d_first_layer_window" \
  "tests/test_gpu_kernels.py::test_conv3d_row_window" "tests/test_gpu_kernels.py::test_conv_first_layer_smallc" \
  tests/test_gpu_model.py -k "3 or first or step" -q -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed" $o/tests.log | tail -3
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" $o/tests.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --dims 3 --per_gpu_batch 8 --steps 5 --warmup 2 > $o/d3.log 2>&1 \
  || { echo "d3 rc=$?"; tail -20 $o/d3.log; exit 1; }
grep '^{' $o/d3.log | cut -c1-160
timeout -k 10 300 python tools/layer_times.py --batch 8 --img 128 --dims 3 --in_channels 4 --reps 3 \
  --out $o/layer_times_3d_b8.md > $o/lt3d.log 2>&1 || { echo "lt3d rc=$?"; tail -20 $o/lt3d.log; exit 1; }
head -3 $o/layer_times_3d_b8.md | tail -1
grep -E "conv1a" $o/layer_times_3d_b8.md | head -4
