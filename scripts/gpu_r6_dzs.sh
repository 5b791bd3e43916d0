#!/bin/bash
# Round 6: norm backward on load in the split consumers (dz_split) -- tests, BN per-launch A/B, benches.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6dzs; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dz_split.py \
  > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_norm_fused.py \
  tests/test_gpu_conv_dw.py > $o/tests_n.log 2>&1 || { echo "norm tests rc=$?"; tail -40 $o/tests_n.log; exit 1; }
tail -1 $o/tests_n.log
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_model.py \
  tests/test_gpu_fp16.py -k "norm or batch or group" > $o/tests_m.log 2>&1 || { echo "model tests rc=$?"; tail -40 $o/tests_m.log; exit 1; }
tail -1 $o/tests_m.log
for v in 0 1; do
  UNET_ENGINE="fwd_streams=1,dz_split=$v" timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 \
    --norm batch --out $o/lt_bn_$v.md > $o/lt_bn_$v.log 2>&1 || { echo "lt bn rc=$?"; tail -20 $o/lt_bn_$v.log; exit 1; }
  head -3 $o/lt_bn_$v.md | tail -1
done
python tools/lt_diff.py $o/lt_bn_0.md $o/lt_bn_1.md 24
for v in 0 1; do
  UNET_ENGINE="dz_split=$v" timeout -k 10 300 python bench.py --norm batch --steps 20 --warmup 5 > $o/bench_bn_$v.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_bn_$v.log; exit 1; }
  tail -1 $o/bench_bn_$v.log | cut -c1-200
done
timeout -k 10 300 python bench.py --norm group --dtype fp16 --steps 20 --warmup 5 > $o/bench_gn.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_gn.log; exit 1; }
tail -1 $o/bench_gn.log | cut -c1-200
