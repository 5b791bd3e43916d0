#!/bin/bash
# Round 5 (re-entry session) evidence: GPU suite on the final tree, every BASELINE config
# (512^2 / 3D at their best batches), per-launch times of the headline and the BN step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
SKIP_FP32=1 bash scripts/gpu_r5_configs.sh "64 128" "8" || exit 1
o=gpurun_out/fin; mkdir -p $o
UNET_ENGINE=fwd_streams=1 timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --norm batch --reps 5 \
  --out $o/layer_times_bn.md > $o/ltbn.log 2>&1 || { echo "ltbn rc=$?"; tail -20 $o/ltbn.log; exit 1; }
head -3 $o/layer_times_bn.md | tail -1
UNET_ENGINE=fwd_streams=1 timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --reps 5 \
  --out $o/layer_times.md > $o/lt.log 2>&1 || { echo "lt rc=$?"; tail -20 $o/lt.log; exit 1; }
head -3 $o/layer_times.md | tail -1
