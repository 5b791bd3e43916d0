#!/bin/bash
# Round 5: fp32 executor (kernel + whole-step tests, CLI), an fp32 bench line, then the
# 3D batch sweep and per-launch times of 512^2 / 3D.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5f32; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_cli.py -v -s --timeout 200 --timeout-method thread \
  > $o/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|worst|Error" $o/tests.log | tail -30
[ $rc -gt 1 ] && { echo "tests crashed rc=$rc"; tail -30 $o/tests.log; exit 1; }
timeout -k 10 300 python bench.py --dtype fp32 --steps 5 --warmup 2 > $o/bench_fp32.log 2>&1 || { echo "fp32 bench rc=$?"; tail -20 $o/bench_fp32.log; exit 1; }
grep '^{' $o/bench_fp32.log | cut -c1-400
bash scripts/gpu_r5_b.sh
