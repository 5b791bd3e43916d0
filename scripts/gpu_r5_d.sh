#!/bin/bash
# Round 5 check D: tests touched this round, headline bench, profile (kernel stats,
# per-launch times, PMC: MFMA / LDS conflicts / bytes), the big-batch configs (chunked
# wgrad), and the upsampling-decoder Dice experiment at the reference's defaults.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5d; mkdir -p $o
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_kernels.py tests/test_gpu_model.py \
  tests/test_gpu_conv_dw.py -q -s --timeout 300 --timeout-method thread > $o/tests.log 2>&1; rc=$?
grep -E "passed|failed|worst" $o/tests.log | tail -8
[ $rc -gt 1 ] && { echo "tests crashed rc=$rc"; tail -30 $o/tests.log; exit 1; }
[ $rc -eq 1 ] && grep -E "^FAILED|Error" $o/tests.log | head -20
timeout -k 10 240 python bench.py > $o/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench.log; exit 1; }
grep '^{' $o/bench.log | cut -c1-200
timeout -k 10 200 python bench.py --dtype fp32 --backend torch --per_gpu_batch 128 --steps 3 --warmup 1 > $o/bench_aten32.log 2>&1 || echo "aten fp32 bench rc=$?"
grep '^{' $o/bench_aten32.log | cut -c1-120
timeout -k 10 200 python bench.py --dtype fp32 --per_gpu_batch 128 --steps 3 --warmup 1 > $o/bench_f32.log 2>&1 || echo "native fp32 bench rc=$?"
grep '^{' $o/bench_f32.log | cut -c1-120
bash scripts/gpu_profile.sh r5 > $o/profile.log 2>&1 || { echo "profile rc=$?"; tail -20 $o/profile.log; exit 1; }
head -30 gpurun_out/prof_r5/pmc_table.md
SKIP_MAIN=1 bash scripts/gpu_r5_configs.sh "128" "16" || echo "configs failed"
timeout -k 10 1500 bash scripts/gpu_r5_ups_dice.sh 200 1 2 3 > $o/dice.log 2>&1 || { echo "dice rc=$?"; tail -20 $o/dice.log; exit 1; }
tail -12 gpurun_out/dice_ups/summary.md
