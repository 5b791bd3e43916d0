#!/bin/bash
# Round 6: bench-shape oracle (forward, weight and data gradients).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6t2; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_shape.py \
  > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -3 $o/tests.log
