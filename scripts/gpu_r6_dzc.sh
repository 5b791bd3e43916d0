#!/bin/bash
# Round 6: dz_split (norm backward on load in the split consumers) + 128-wide wgrad halo-row
# carry -- tests, per-launch A/B, benches.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6dzc; mkdir -p $o
t() { timeout -k 10 $1 python -u -m pytest -x -v --timeout ${3:-120} --timeout-method thread "${@:4}" > $o/$2.log 2>&1 || { echo "$2 rc=$?"; tail -40 $o/$2.log; exit 1; }; tail -1 $o/$2.log; }
t 600 t_dz 120 tests/test_gpu_dz_split.py
t 600 t_wg 120 tests/test_gpu_kernels.py -k "wgrad"
t 600 t_nf 120 tests/test_gpu_norm_fused.py tests/test_gpu_conv_dw.py tests/test_gpu_bounds.py
t 900 t_m 300 tests/test_gpu_model.py tests/test_gpu_fp16.py -k "norm or batch or group or 3d or dims"
lt() { UNET_ENGINE="fwd_streams=1$1" timeout -k 10 400 python tools/layer_times.py ${@:3} --out $o/$2.md > $o/$2.log 2>&1 || { echo "lt $2 rc=$?"; tail -20 $o/$2.log; exit 1; }; head -3 $o/$2.md | tail -1; }
lt ",dz_split=0" lt_bn_0 --batch 1024 --img 128 --norm batch
lt "" lt_bn_1 --batch 1024 --img 128 --norm batch
python tools/lt_diff.py $o/lt_bn_0.md $o/lt_bn_1.md 24
lt "" lt_3d --batch 8 --img 128 --dims 3
python tools/lt_diff.py profiles/r6_layer_times_3d_b8.md $o/lt_3d.md 10
lt "" lt_head --batch 1024 --img 128
python tools/lt_diff.py profiles/r6_layer_times.md $o/lt_head.md 10
b() { timeout -k 10 300 python bench.py --steps 20 --warmup 5 "${@:2}" > $o/$1.log 2>&1 || { echo "bench $1 rc=$?"; tail -20 $o/$1.log; exit 1; }; tail -1 $o/$1.log | cut -c1-160; }
UNET_ENGINE="dz_split=0" b bench_bn_0 --norm batch
b bench_bn_1 --norm batch
b bench_gn --norm group --dtype fp16
b bench_3d --dims 3 --per_gpu_batch 8
b bench
