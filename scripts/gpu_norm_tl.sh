#!/bin/bash
# Kernel timelines + bench lines of the normalised configs (BN bf16, GN fp16), after
# the fused-norm GPU tests:  bash scripts/gpu_norm_tl.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-cur}
o=gpurun_out/tl_$tag
rm -rf $o; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_norm_fused.py tests/test_gpu_kernels.py tests/test_gpu_fp16.py -k "norm or fp16 or group or head" -x -q --timeout 120 --timeout-method thread \
  > $o/pytest.log 2>&1 || { tail -20 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for n in bn gn16; do
  a="--norm batch"; [ $n = gn16 ] && a="--norm group --dtype fp16"
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $o/$n -o run -- \
    python bench.py --steps 4 --warmup 2 $a > $o/$n.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --norm batch --steps 10 --warmup 3 > $o/bench.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --dtype fp16 --norm group --steps 10 --warmup 3 >> $o/bench.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' $o/bench.log
