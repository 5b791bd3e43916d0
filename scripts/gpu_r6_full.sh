#!/bin/bash
# Round 6: whole GPU suite, then head_wsum / XF1-dropout per-launch checks and benches.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6full; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/gpu_suite.log 2>&1 || { echo "suite rc=$?"; tail -40 $o/gpu_suite.log; exit 1; }
tail -2 $o/gpu_suite.log
lt() { UNET_ENGINE="fwd_streams=1$1" timeout -k 10 400 python tools/layer_times.py ${@:3} --out $o/$2.md > $o/$2.log 2>&1 || { echo "lt $2 rc=$?"; tail -20 $o/$2.log; exit 1; }; head -3 $o/$2.md | tail -1; }
lt ",head_wsum=0" lt_h0 --batch 1024 --img 128
lt "" lt_h1 --batch 1024 --img 128
python tools/lt_diff.py $o/lt_h0.md $o/lt_h1.md 6
lt "" lt_bn --batch 1024 --img 128 --norm batch
python tools/lt_diff.py profiles/r6_layer_times_bn.md $o/lt_bn.md 12
b() { timeout -k 10 300 python bench.py --steps 20 --warmup 5 "${@:2}" > $o/$1.log 2>&1 || { echo "bench $1 rc=$?"; tail -20 $o/$1.log; exit 1; }; tail -1 $o/$1.log | cut -c1-150; }
UNET_ENGINE="head_wsum=0" b bench_h0
b bench_h1
UNET_ENGINE="head_wsum=0" b bench_h0b
b bench_h1b
b bench_bn --norm batch
b bench_gn --norm group --dtype fp16
