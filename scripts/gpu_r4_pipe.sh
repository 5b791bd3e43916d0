#!/bin/bash
# Pipelined 8-wave window: bit-exactness vs the 4-wave window, the kernel / model suites,
# then a same-box interleaved A/B of the headline step (conv_pipe 0 / 1).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_pipe.py > gpurun_out/pipe_tests.log 2>&1 || { echo "pipe tests rc=$?"; tail -40 gpurun_out/pipe_tests.log; exit 1; }
tail -2 gpurun_out/pipe_tests.log
timeout -k 10 600 $T tests/test_gpu_kernels.py tests/test_gpu_norm_fused.py tests/test_gpu_tconv_fused.py > gpurun_out/pipe_ktests.log 2>&1 || { echo "kernel tests rc=$?"; tail -40 gpurun_out/pipe_ktests.log; exit 1; }
tail -2 gpurun_out/pipe_ktests.log
bash scripts/gpu_ab_env.sh UNET_ENGINE conv_pipe=0 conv_pipe=1 3 || exit $?
