#!/bin/bash
# Window kernels on segmented rows (512x512) and 3D: kernel parity tests, whole-step
# parity, then benches + per-launch layer times of the 3 configs.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "segmented or conv3d or wgrad3d or row_window" > gpurun_out/tests_winext.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_model.py \
  -k "matches_reference" > gpurun_out/tests_model.log 2>&1 || exit $?
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 180 python bench.py --steps 10 --warmup 3 --img_size 512 --in_channels 1 --per_gpu_batch 16 \
  > gpurun_out/bench_512.log 2>&1 || exit $?
timeout -k 10 180 python bench.py --steps 10 --warmup 3 --dims 3 --per_gpu_batch 2 > gpurun_out/bench_3d.log 2>&1 || exit $?
timeout -k 10 180 python tools/layer_times.py --batch 16 --img 512 --in_channels 1 --out gpurun_out/layer_times_512.md \
  > /dev/null 2>&1 || exit $?
timeout -k 10 180 python tools/layer_times.py --batch 2 --img 128 --dims 3 --out gpurun_out/layer_times_3d.md \
  > /dev/null 2>&1 || exit $?
grep -h metric gpurun_out/bench.log gpurun_out/bench_512.log gpurun_out/bench_3d.log
