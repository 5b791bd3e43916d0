#!/bin/bash
# head sums in the forward: tests + A/B; level-3 composite with the chained wgrad; 512^2 check
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q --timeout 150 \
  --timeout-method thread > gpurun_out/r3h_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r3h_tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ab_env.sh UNET_HEAD_SUMS 0 1 3 || exit $?
bash scripts/gpu_ab_env.sh UNET_TCONV_FUSED 2 3 2 || exit $?
bash scripts/gpu_ab_env.sh UNET_TCONV_FWD 0 1 1 --img_size 512 --in_channels 1 --per_gpu_batch 16 --steps 10 --warmup 3
