#!/bin/bash
# Persistent tconv-on-load window with the statistics epilogue (normalised configs' conv9a):
# kernel tests, the norm model tests, then a same-box A/B against the tree before it (ab_old)
# on the BatchNorm and GroupNorm fp16 benches.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tconv_fused.py tests/test_gpu_model.py tests/test_gpu_norm_fused.py tests/test_gpu_fp16.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pfust_tests.log 2>&1 || { tail -30 gpurun_out/pfust_tests.log; exit 1; }
tail -1 gpurun_out/pfust_tests.log
UNET_ENGINE=fwd_streams=1 timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --norm batch --reps 5 \
  --out gpurun_out/layer_times_bn_pfust.md > gpurun_out/ltbn.log 2>&1 || { echo "ltbn rc=$?"; tail -20 gpurun_out/ltbn.log; exit 1; }
head -3 gpurun_out/layer_times_bn_pfust.md | tail -1
grep "fwd:conv9a" gpurun_out/layer_times_bn_pfust.md
bash scripts/gpu_ab_tree.sh ab_old 3 --norm batch --steps 10 --warmup 3 || exit 1
mv gpurun_out/abt gpurun_out/abt_bn2
bash scripts/gpu_ab_tree.sh ab_old 2 --norm group --dtype fp16 --steps 10 --warmup 3 || exit 1
mv gpurun_out/abt gpurun_out/abt_gn2
