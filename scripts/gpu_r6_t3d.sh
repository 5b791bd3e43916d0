#!/bin/bash
# Round 6: 3D defaults (win_cp3=2, wg_pf=1) -- window / model tests, 3D bench.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6t3d; mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_win_cp.py tests/test_gpu_model.py tests/test_gpu_bounds.py -k "3d or dims or cp or D3 or bound" > $o/t.log 2>&1 || { echo "t rc=$?"; tail -40 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 300 python bench.py --dims 3 --steps 6 --warmup 2 > $o/b.log 2>&1 || { echo "b rc=$?"; tail -20 $o/b.log; exit 1; }
tail -1 $o/b.log | cut -c1-120
