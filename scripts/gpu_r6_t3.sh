#!/bin/bash
# Round 6: 3D tconv forward window -- kernel tests, 3D model tests, 3D bench + layer table.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6t3; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread "tests/test_gpu_kernels.py" \
  -k "tconv or conv3d" > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_model.py \
  > $o/tests_model.log 2>&1 || { echo "model tests rc=$?"; tail -40 $o/tests_model.log; exit 1; }
tail -2 $o/tests_model.log
timeout -k 10 300 python bench.py --dims 3 --per_gpu_batch 8 --steps 5 --warmup 2 > $o/d3.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/d3.log; exit 1; }
grep '^{' $o/d3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('d3 b8', d['value'], d['ms_per_step'])"
UNET_ENGINE="fwd_streams=1" timeout -k 10 400 python tools/layer_times.py --batch 8 --img 128 --dims 3 \
  --out $o/lt_3d_b8.md > $o/lt_3d.log 2>&1 || { echo "lt 3d rc=$?"; tail -20 $o/lt_3d.log; exit 1; }
head -3 $o/lt_3d_b8.md
