#!/bin/bash
# chained consumer wgrad (UNET_TCONV_FWD=1 default): tests, then same-box A/B 0 vs 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tconv_fused.py tests/test_gpu_model.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r3c_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash scripts/gpu_ab_env.sh UNET_TCONV_FWD 0 1 3
