#!/bin/bash
# Pipelined 8-wave windows (conv_pipe.h, wgrad_pipe.hip): equivalence vs the 4-wave
# windows, the kernel / model suites, then same-box interleaved A/Bs of the headline step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_pipe.py > gpurun_out/pipe_tests.log 2>&1 || { echo "pipe tests rc=$?"; tail -40 gpurun_out/pipe_tests.log; exit 1; }
tail -2 gpurun_out/pipe_tests.log
timeout -k 10 200 python bench.py > gpurun_out/pipe_bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/pipe_bench.log; exit 1; }
grep metric gpurun_out/pipe_bench.log
bash scripts/gpu_ab_env.sh UNET_ENGINE conv_pipe=0,wgrad_pipe=0 conv_pipe=1,wgrad_pipe=1 2 || exit $?
bash scripts/gpu_ab_env.sh UNET_ENGINE wgrad_pipe=0 wgrad_pipe=1 1 || exit $?
timeout -k 10 900 $T tests/test_gpu_kernels.py tests/test_gpu_norm_fused.py tests/test_gpu_tconv_fused.py tests/test_gpu_model.py > gpurun_out/pipe_ktests.log 2>&1 || { echo "kernel/model tests rc=$?"; tail -40 gpurun_out/pipe_ktests.log; exit 1; }
tail -2 gpurun_out/pipe_ktests.log
