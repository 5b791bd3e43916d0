#!/bin/bash
# Register-prefetched chunk loop (conv_win.h PF): bit-identity + whole-step tests, per-launch
# A/B (win_pf 0 / 1), then a same-box interleaved bench A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
( while sleep 60; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -v -s \
  -k "prefetch or row_window or native_step or concat" --timeout 300 --timeout-method thread > gpurun_out/r4_pf_tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -40 gpurun_out/r4_pf_tests.log; exit 1; }
tail -3 gpurun_out/r4_pf_tests.log
bash scripts/gpu_r4_lt.sh "win_pf=0" "win_pf=1" || exit 1
bash scripts/gpu_ab_env.sh UNET_ENGINE win_pf=0 win_pf=1 3
