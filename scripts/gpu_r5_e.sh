#!/bin/bash
# Round 5 check E: the GPU suite after the XF 5 (tconv on load) u-store and epilogue-staging
# conflict fixes, the float64-oracle fp32
# step test, headline bench + profile, per-launch times of the 512^2 and 3D configs
# (limiting kernels), and the upsampling-decoder Dice seeds 2-3.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5e; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed|worst" $o/tests.log | tail -8
[ $rc -gt 1 ] && { echo "tests crashed rc=$rc"; tail -30 $o/tests.log; exit 1; }
[ $rc -eq 1 ] && grep -E "^FAILED|Error" $o/tests.log | head -20
timeout -k 10 240 python bench.py > $o/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench.log; exit 1; }
grep '^{' $o/bench.log | cut -c1-200
bash scripts/gpu_profile.sh r5e > $o/profile.log 2>&1 || { echo "profile rc=$?"; tail -20 $o/profile.log; exit 1; }
grep -E "conv9a|step" gpurun_out/prof_r5e/layer_times.md | head -5
grep -E "ELEMENT|kernel \||1, 0, 5>" gpurun_out/prof_r5e/pmc_table.md | head -4
timeout -k 10 300 python tools/layer_times.py --batch 32 --img 512 --in_channels 1 --reps 5 \
  --out gpurun_out/prof_r5e/layer_times_s512_b32.md > $o/lt512.log 2>&1 || { echo "lt512 rc=$?"; tail -20 $o/lt512.log; exit 1; }
head -4 gpurun_out/prof_r5e/layer_times_s512_b32.md
timeout -k 10 300 python tools/layer_times.py --batch 8 --img 128 --dims 3 --in_channels 4 --reps 3 \
  --out gpurun_out/prof_r5e/layer_times_3d_b8.md > $o/lt3d.log 2>&1 || { echo "lt3d rc=$?"; tail -20 $o/lt3d.log; exit 1; }
head -4 gpurun_out/prof_r5e/layer_times_3d_b8.md
timeout -k 10 900 bash scripts/gpu_r5_ups_dice.sh 200 2 3 > $o/dice.log 2>&1 || { echo "dice rc=$?"; tail -20 $o/dice.log; exit 1; }
tail -12 gpurun_out/dice_ups/summary.md
