#!/bin/bash
# Round 6: 3D head_wsum (head_wsum=2) -- numerics vs head_bwd, per-launch times and the 3D bench A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6hws3d; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -k "head_wsum" -x -v --timeout 120 --timeout-method thread > $o/test.log 2>&1 || { echo "test rc=$?"; tail -40 $o/test.log; exit 1; }
tail -2 $o/test.log
lt() { UNET_ENGINE="fwd_streams=1$1" timeout -k 10 400 python tools/layer_times.py ${@:3} --out $o/$2.md > $o/$2.log 2>&1 || { echo "lt $2 rc=$?"; tail -20 $o/$2.log; exit 1; }; head -3 $o/$2.md | tail -1; }
lt "" lt_1 --batch 8 --img 128 --dims 3
lt ",head_wsum=2" lt_2 --batch 8 --img 128 --dims 3
python tools/lt_diff.py $o/lt_1.md $o/lt_2.md 10
b() { timeout -k 10 300 python bench.py "${@:2}" > $o/$1.log 2>&1 || { echo "bench $1 rc=$?"; tail -20 $o/$1.log; exit 1; }; tail -1 $o/$1.log | cut -c1-110; }
for r in 1 2; do
  b b1 --dims 3 --steps 6 --warmup 2
  UNET_ENGINE="head_wsum=2" b b2 --dims 3 --steps 6 --warmup 2
done
