#!/bin/bash
# z-prefetch check: norm-fused kernel tests, norm step tests, BN / GN per-launch times, benches
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/zpre; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_norm_fused.py \
  tests/test_gpu_model.py -k "norm or Norm" > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
bash scripts/gpu_r4_bn_lt.sh zpre || exit 1
for a in "--norm batch" "--norm group --dtype fp16"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $a > $o/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/bench.log; exit 1; }
  tail -1 $o/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['ms_per_step'])"
done
