#!/bin/bash
# Round 6: prefetching 128-wide window weight gradient (wg_pf) -- tests, per-launch A/B, benches.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6wpf; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad" > $o/t.log 2>&1 || { echo "t rc=$?"; tail -40 $o/t.log; exit 1; }
tail -1 $o/t.log
lt() { UNET_ENGINE="fwd_streams=1$1" timeout -k 10 400 python tools/layer_times.py ${@:3} --out $o/$2.md > $o/$2.log 2>&1 || { echo "lt $2 rc=$?"; tail -20 $o/$2.log; exit 1; }; head -3 $o/$2.md | tail -1; }
lt ",wg_pf=0" lt3_0 --batch 8 --img 128 --dims 3
lt ",wg_pf=1" lt3_1 --batch 8 --img 128 --dims 3
python tools/lt_diff.py $o/lt3_0.md $o/lt3_1.md 8
lt ",wg_pf=0" lth_0 --batch 1024 --img 128
lt ",wg_pf=2" lth_2 --batch 1024 --img 128
python tools/lt_diff.py $o/lth_0.md $o/lth_2.md 6
b() { timeout -k 10 300 python bench.py "${@:2}" > $o/$1.log 2>&1 || { echo "bench $1 rc=$?"; tail -20 $o/$1.log; exit 1; }; tail -1 $o/$1.log | cut -c1-130; }
UNET_ENGINE="wg_pf=0" b b3_0 --dims 3 --steps 6 --warmup 2
UNET_ENGINE="wg_pf=1" b b3_1 --dims 3 --steps 6 --warmup 2
UNET_ENGINE="wg_pf=0" b bh_0 --steps 20 --warmup 5
UNET_ENGINE="wg_pf=2" b bh_2 --steps 20 --warmup 5
