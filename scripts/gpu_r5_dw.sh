#!/bin/bash
# Round 5: fused data + weight gradient (conv_dw.hip) -- kernel tests, the whole-step
# parity tests, an interleaved bench A/B (dw_fuse 0 / 1) and per-launch times.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r5dw; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_dw.py tests/test_gpu_f32.py -q --timeout 120 --timeout-method thread \
  > $o/tests.log 2>&1 || { echo "dw/f32 tests rc=$?"; grep -E "FAILED|Error|assert" $o/tests.log | head -30; }
tail -2 $o/tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread \
  > $o/model.log 2>&1 || { echo "model tests rc=$?"; tail -40 $o/model.log; exit 1; }
tail -2 $o/model.log
for r in 1 2 3; do
  for v in 0 1; do
    UNET_ENGINE="dw_fuse=$v" timeout -k 10 200 python bench.py > $o/b_${v}_$r.log 2>&1 || { echo "bench rc=$?"; tail $o/b_${v}_$r.log; exit 1; }
    python -c "import json,sys; r=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('dw_fuse=$v round $r', r['value'], r['ms_per_step'])" $o/b_${v}_$r.log
  done
done
UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 --out $o/lt_dw.md > $o/lt.log 2>&1 || { echo "lt rc=$?"; tail -20 $o/lt.log; exit 1; }
head -3 $o/lt_dw.md
grep "conv1" $o/lt_dw.md
