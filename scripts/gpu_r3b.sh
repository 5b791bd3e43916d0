#!/bin/bash
# composite forward tests, then same-box A/Bs: epilogue prefetch (tree A/B vs ab_old) and
# the composite forward (UNET_TCONV_FWD 0 / 1)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_tconv_fused.py tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r3b_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash scripts/gpu_ab_tree.sh ab_old 3 || exit $?
bash scripts/gpu_ab_env.sh UNET_TCONV_FWD 0 1 2
