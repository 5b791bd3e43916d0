#!/bin/bash
# Round 6: bench-shape oracle (forward, weight and data gradients).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6t2; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_shape.py \
  > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -3 $o/tests.log
o2=gpurun_out/r6f32; mkdir -p $o2
for b in 128 256 512; do
  timeout -k 10 300 python bench.py --dtype fp32 --per_gpu_batch $b --steps 5 --warmup 2 > $o2/b$b.log 2>&1 || { echo "fp32 b$b rc=$?"; tail -20 $o2/b$b.log; exit 1; }
  grep '^{' $o2/b$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fp32 b$b', d['value'], d['ms_per_step'])"
done
