#!/bin/bash
# Round-5 baseline on one box: headline bench + per-launch times of the current tree.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5base
timeout -k 10 240 python bench.py > gpurun_out/r5base/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/r5base/bench.log; exit 1; }
grep metric gpurun_out/r5base/bench.log
UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --out gpurun_out/r5base/lt.md > gpurun_out/r5base/lt.log 2>&1 || { echo "lt rc=$?"; tail -20 gpurun_out/r5base/lt.log; exit 1; }
head -3 gpurun_out/r5base/lt.md
