#!/bin/bash
# Round 6: BatchNorm skip source normalised on load (skip_onload) -- tests, per-launch A/B, bench.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6sko; mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_norm_fused.py tests/test_gpu_win_pf.py -k "skip_onload or batch or norm or pfu or onload" > $o/t.log 2>&1 || { echo "t rc=$?"; tail -40 $o/t.log; exit 1; }
tail -1 $o/t.log
lt() { UNET_ENGINE="fwd_streams=1$1" timeout -k 10 400 python tools/layer_times.py ${@:3} --out $o/$2.md > $o/$2.log 2>&1 || { echo "lt $2 rc=$?"; tail -20 $o/$2.log; exit 1; }; head -3 $o/$2.md | tail -1; }
lt ",skip_onload=0" lt_0 --batch 1024 --img 128 --norm group --dtype fp16
lt "" lt_1 --batch 1024 --img 128 --norm group --dtype fp16
python tools/lt_diff.py $o/lt_0.md $o/lt_1.md 8
b() { timeout -k 10 300 python bench.py "${@:2}" > $o/$1.log 2>&1 || { echo "bench $1 rc=$?"; tail -20 $o/$1.log; exit 1; }; echo "$1 $(grep -o '"value": [0-9.]*' $o/$1.log)"; }
UNET_ENGINE="skip_onload=0" b b0 --norm group --dtype fp16 --steps 12 --warmup 4
b b1 --norm group --dtype fp16 --steps 12 --warmup 4
UNET_ENGINE="skip_onload=0" b b0b --norm group --dtype fp16 --steps 12 --warmup 4
b b1b --norm group --dtype fp16 --steps 12 --warmup 4
