#!/bin/bash
# Round 6: head_wsum with the hardware reciprocal -- per-launch A/B + benches.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6hws2; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py -k "head_wsum" > $o/t.log 2>&1 || { echo "t rc=$?"; tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
lt() { UNET_ENGINE="fwd_streams=1$1" timeout -k 10 400 python tools/layer_times.py ${@:3} --out $o/$2.md > $o/$2.log 2>&1 || { echo "lt $2 rc=$?"; tail -20 $o/$2.log; exit 1; }; head -3 $o/$2.md | tail -1; }
lt ",head_wsum=0" lt_h0 --batch 1024 --img 128
lt "" lt_h1 --batch 1024 --img 128
python tools/lt_diff.py $o/lt_h0.md $o/lt_h1.md 6
b() { timeout -k 10 300 python bench.py --steps 20 --warmup 5 "${@:2}" > $o/$1.log 2>&1 || { echo "bench $1 rc=$?"; tail -20 $o/$1.log; exit 1; }; tail -1 $o/$1.log | cut -c1-150; }
UNET_ENGINE="head_wsum=0" b bench_h0
b bench_h1
UNET_ENGINE="head_wsum=0" b bench_h0b
b bench_h1b
