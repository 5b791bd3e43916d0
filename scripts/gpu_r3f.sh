#!/bin/bash
# composite tconv backward in norm mode: tests, then BN / GN fp16 same-box A/Bs
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_norm_fused.py tests/test_gpu_tconv_fused.py \
  -x -q --timeout 150 --timeout-method thread > gpurun_out/r3f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r3f_tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ab_env.sh UNET_TCONV_FUSED 0 2 2 --norm batch --steps 10 --warmup 3 || exit $?
bash scripts/gpu_ab_env.sh UNET_TCONV_FUSED 0 2 2 --norm group --dtype fp16 --steps 10 --warmup 3
