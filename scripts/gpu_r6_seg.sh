#!/bin/bash
# Round 6: segmented-row conv_dw -- kernel tests, 512^2 step tests, 512^2 benches + layer table.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6seg; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv_dw.py \
  tests/test_gpu_bounds.py tests/test_gpu_model.py > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for b in 32 64; do
  timeout -k 10 300 python bench.py --img_size 512 --in_channels 1 --per_gpu_batch $b --steps 8 --warmup 3 > $o/s512_b$b.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/s512_b$b.log; exit 1; }
  grep '^{' $o/s512_b$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('s512 b$b', d['value'], d['ms_per_step'])"
done
UNET_ENGINE="fwd_streams=1" timeout -k 10 300 python tools/layer_times.py --batch 32 --img 512 --in_channels 1 \
  --out $o/lt_s512_b32.md > $o/lt_s512.log 2>&1 || { echo "lt 512 rc=$?"; tail -20 $o/lt_s512.log; exit 1; }
head -3 $o/lt_s512_b32.md
