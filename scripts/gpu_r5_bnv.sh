#!/bin/bash
# 16-byte phase-1 loads in the BatchNorm statistics kernel: direct kernel tests, the norm
# model tests, BN per-launch times, same-box A/B against the tree before it (ab_old).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_norm_fused.py tests/test_gpu_model.py tests/test_gpu_fp16.py tests/test_gpu_kernels.py -k "norm or stats or fp16" -x -q --timeout 120 --timeout-method thread > gpurun_out/bnv_tests.log 2>&1 || { tail -30 gpurun_out/bnv_tests.log; exit 1; }
tail -1 gpurun_out/bnv_tests.log
UNET_ENGINE=fwd_streams=1 timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --norm batch --reps 5 \
  --out gpurun_out/layer_times_bn_bnv.md > gpurun_out/ltbn.log 2>&1 || { echo "ltbn rc=$?"; tail -20 gpurun_out/ltbn.log; exit 1; }
head -3 gpurun_out/layer_times_bn_bnv.md | tail -1
grep -E "^\| bnfin" gpurun_out/layer_times_bn_bnv.md
bash scripts/gpu_ab_tree.sh ab_old 3 --norm batch --steps 10 --warmup 3 || exit 1
mv gpurun_out/abt gpurun_out/abt_bn3
