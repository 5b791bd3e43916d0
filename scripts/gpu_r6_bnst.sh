#!/bin/bash
# Round 6: bn_stats_fused with 16-byte loads -- norm tests, BN per-launch table, BN / GN fp16 bench.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6bnst; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_norm_fused.py \
  > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_model.py \
  -k "norm or batch or group" > $o/tests_m.log 2>&1 || { echo "model tests rc=$?"; tail -40 $o/tests_m.log; exit 1; }
tail -1 $o/tests_m.log
UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --norm batch \
  --out $o/lt_bn.md > $o/lt_bn.log 2>&1 || { echo "lt bn rc=$?"; tail -20 $o/lt_bn.log; exit 1; }
head -3 $o/lt_bn.md | tail -1
grep bnfin $o/lt_bn.md | awk -F'|' '{s+=$4} END {print "bnfin total", s}'
python tools/lt_diff.py profiles/r6_layer_times_bn.md $o/lt_bn.md 12
timeout -k 10 300 python bench.py --norm batch --steps 20 --warmup 5 > $o/bench_bn.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_bn.log; exit 1; }
tail -1 $o/bench_bn.log
timeout -k 10 300 python bench.py --norm group --dtype fp16 --steps 20 --warmup 5 > $o/bench_gn.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench_gn.log; exit 1; }
tail -1 $o/bench_gn.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $o/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench.log; exit 1; }
tail -1 $o/bench.log
