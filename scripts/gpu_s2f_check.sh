#!/bin/bash
# Composite transposed-conv forward: kernel + model tests, then a same-box A/B of the
# headline bench (UNET_TCONV_FWD 0 / 1).  A test step that ends other than pass /
# assertion failure stops the script.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tconv_fused.py tests/test_gpu_model.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/s2f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/s2f_tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ab_env.sh UNET_TCONV_FWD 0 1 ${ROUNDS:-2}
