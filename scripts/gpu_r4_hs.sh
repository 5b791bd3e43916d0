#!/bin/bash
# Head-gradient sums from the fused-head forward: kernel + whole-step tests, then a same-box
# interleaved A/B of the headline bench (UNET_ENGINE head_sums = 0 / 1).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
( while sleep 60; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -v -s \
  -k "head or native_step or first_layer" --timeout 300 --timeout-method thread > gpurun_out/r4_hs_tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -40 gpurun_out/r4_hs_tests.log; exit 1; }
tail -3 gpurun_out/r4_hs_tests.log
bash scripts/gpu_ab_env.sh UNET_ENGINE head_sums=0 head_sums=1 3
