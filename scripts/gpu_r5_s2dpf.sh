#!/bin/bash
# Composite transposed-conv weight gradient with the next window prefetched into registers
# (engine option s2d_pf): bit-identity tests, per-launch times, same-box step A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tconv_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s2dpf_tests.log 2>&1 || { tail -30 gpurun_out/s2dpf_tests.log; exit 1; }
tail -1 gpurun_out/s2dpf_tests.log
for v in 0 1; do
  UNET_ENGINE=fwd_streams=1,s2d_pf=$v timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --reps 5 \
    --out gpurun_out/lt_s2dpf_$v.md > gpurun_out/lt_s2dpf_$v.log 2>&1 || { echo "lt rc=$?"; tail -20 gpurun_out/lt_s2dpf_$v.log; exit 1; }
  echo "s2d_pf=$v"; grep -E "wgrad:transConv" gpurun_out/lt_s2dpf_$v.md
done
bash scripts/gpu_ab_env.sh UNET_ENGINE s2d_pf=0 s2d_pf=1 3 || exit 1
