#!/bin/bash
# Round 6: 3D tail halves (tail3) -- numerics, per-launch times and the 3D bench A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6tail3; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -k "tail3" -x -v --timeout 120 --timeout-method thread > $o/test.log 2>&1 || { echo "test rc=$?"; tail -40 $o/test.log; exit 1; }
tail -2 $o/test.log
b() { timeout -k 10 300 python bench.py "${@:2}" > $o/$1.log 2>&1 || { echo "bench $1 rc=$?"; tail -20 $o/$1.log; exit 1; }; tail -1 $o/$1.log | cut -c1-110; }
for r in 1 2 3; do
  b b0 --dims 3 --steps 6 --warmup 2
  UNET_ENGINE="tail3=1" b b1 --dims 3 --steps 6 --warmup 2
done
