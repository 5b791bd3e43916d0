#!/bin/bash
# Transposed conv on load (conv_win.h XF 5) + multi-window first layer: kernel and
# whole-step tests, per-launch A/B against ab_base/, then a same-box interleaved A/B of
# the headline bench (UNET_ENGINE tconv_onload = 0 / 1 / 2: deepest level formed on load).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
( while sleep 60; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_tconv_fused.py tests/test_gpu_model.py tests/test_gpu_kernels.py \
  -m gpu -x -v -s -k "onload or first_layer or native_step_matches_reference_at_shipped_shape" \
  --timeout 300 --timeout-method thread > gpurun_out/r4_ut_tests.log 2>&1 || { echo "tests rc=$?"; tail -40 gpurun_out/r4_ut_tests.log; exit 1; }
tail -3 gpurun_out/r4_ut_tests.log
bash scripts/gpu_r4_lt_tree.sh || exit 1
for r in 1 2 3; do
  for v in 0 1 2; do
    UNET_ENGINE=tconv_onload=$v timeout -k 10 200 python bench.py > gpurun_out/ab/ut_${v}_$r.log 2>&1 || exit 1
    python -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('tconv_onload=$v round $r', r['value'], r['ms_per_step'])" gpurun_out/ab/ut_${v}_$r.log
  done
done
