#!/bin/bash
# Round 6: 3D level-1 chunk-pipelined window (win_cp=2) re-measured on the current tree.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6cp3; mkdir -p $o
lt() { UNET_ENGINE="fwd_streams=1$1" timeout -k 10 400 python tools/layer_times.py ${@:3} --out $o/$2.md > $o/$2.log 2>&1 || { echo "lt $2 rc=$?"; tail -20 $o/$2.log; exit 1; }; head -3 $o/$2.md | tail -1; }
lt "" lt_1 --batch 8 --img 128 --dims 3
lt ",win_cp=2" lt_2 --batch 8 --img 128 --dims 3
python tools/lt_diff.py $o/lt_1.md $o/lt_2.md 12
b() { timeout -k 10 300 python bench.py "${@:2}" > $o/$1.log 2>&1 || { echo "bench $1 rc=$?"; tail -20 $o/$1.log; exit 1; }; tail -1 $o/$1.log | cut -c1-110; }
b b1 --dims 3 --steps 6 --warmup 2
UNET_ENGINE="win_cp=2" b b2 --dims 3 --steps 6 --warmup 2
b b1b --dims 3 --steps 6 --warmup 2
UNET_ENGINE="win_cp=2" b b2b --dims 3 --steps 6 --warmup 2
