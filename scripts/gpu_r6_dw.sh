#!/bin/bash
# Round 6: fused dgrad + wgrad with the norm backward on load -- kernel tests, then BN / GN benches.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6dw; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv_dw.py \
  tests/test_gpu_norm_fused.py tests/test_gpu_model.py > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $o/tests.log; exit 1; }
tail -3 $o/tests.log
for cfg in "bn:--norm batch" "gn16:--norm group --dtype fp16" "headline:"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 $args > $o/$tag.log 2>&1 || { echo "bench $tag rc=$?"; tail -20 $o/$tag.log; exit 1; }
  grep '^{' $o/$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'])"
done
UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --norm batch \
  --out $o/lt_bn.md > $o/lt_bn.log 2>&1 || { echo "lt rc=$?"; tail -20 $o/lt_bn.log; exit 1; }
head -3 $o/lt_bn.md
UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 \
  --out $o/lt_head.md > $o/lt_head.log 2>&1 || { echo "lt rc=$?"; tail -20 $o/lt_head.log; exit 1; }
head -3 $o/lt_head.md
