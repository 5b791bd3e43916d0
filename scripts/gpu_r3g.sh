#!/bin/bash
# 8x8 image window with normalisation epilogues: tests, then BN A/B vs ab_old (HEAD)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_norm_fused.py -x -q \
  --timeout 150 --timeout-method thread > gpurun_out/r3g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r3g_tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ab_tree.sh ab_old 2 --norm batch --steps 10 --warmup 3
