#!/bin/bash
# Round 6: Mask gradients from forward sums (head_wsum), norm-head loads -- tests, A/B, benches.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6hws; mkdir -p $o
t() { timeout -k 10 $1 python -u -m pytest -x -v --timeout ${3:-120} --timeout-method thread "${@:4}" > $o/$2.log 2>&1 || { echo "$2 rc=$?"; tail -40 $o/$2.log; exit 1; }; tail -1 $o/$2.log; }
t 900 t_m 300 tests/test_gpu_model.py -k "head or native_step or hip_graph"
t 600 t_k 120 tests/test_gpu_kernels.py tests/test_gpu_win_pf.py tests/test_gpu_bounds.py -k "head or pf or bound or fused"
lt() { UNET_ENGINE="fwd_streams=1$1" timeout -k 10 400 python tools/layer_times.py ${@:3} --out $o/$2.md > $o/$2.log 2>&1 || { echo "lt $2 rc=$?"; tail -20 $o/$2.log; exit 1; }; head -3 $o/$2.md | tail -1; }
lt ",head_wsum=0" lt_h0 --batch 1024 --img 128
lt "" lt_h1 --batch 1024 --img 128
python tools/lt_diff.py $o/lt_h0.md $o/lt_h1.md 10
b() { timeout -k 10 300 python bench.py --steps 20 --warmup 5 "${@:2}" > $o/$1.log 2>&1 || { echo "bench $1 rc=$?"; tail -20 $o/$1.log; exit 1; }; tail -1 $o/$1.log | cut -c1-150; }
UNET_ENGINE="head_wsum=0" b bench_h0
b bench_h1
UNET_ENGINE="head_wsum=0" b bench_h0b
b bench_h1b
b bench_bn --norm batch
