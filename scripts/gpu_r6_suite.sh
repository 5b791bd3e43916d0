#!/bin/bash
# Round 6: whole GPU suite + smoke on the current tree, then the 3D configs.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6suite; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_suite.log 2>&1 || { echo "suite rc=$?"; tail -40 $o/gpu_suite.log; exit 1; }
tail -2 $o/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $o/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
b() { timeout -k 10 300 python bench.py "${@:2}" > $o/$1.log 2>&1 || { echo "bench $1 rc=$?"; tail -20 $o/$1.log; exit 1; }; tail -1 $o/$1.log | cut -c1-130; }
b d3_b8 --dims 3 --per_gpu_batch 8 --steps 5 --warmup 2
b d3_b16 --dims 3 --per_gpu_batch 16 --steps 5 --warmup 2
b headline --steps 20 --warmup 5
