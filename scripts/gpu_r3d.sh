#!/bin/bash
# 8x8 image-window conv: kernel + model tests, then a same-box tree A/B vs ab_old (HEAD)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r3d_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r3d_tests.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_ab_tree.sh ab_old 3
