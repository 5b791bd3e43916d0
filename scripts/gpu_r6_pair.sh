#!/bin/bash
# Round 6: wave-pair window weight gradients and 3D head-on-load -- tests, then per-launch A/B.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6pair; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "wgrad" > $o/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_model.py \
  -k "head_onload or native_step_matches_reference" > $o/tests_m.log 2>&1 || { echo "model tests rc=$?"; tail -40 $o/tests_m.log; exit 1; }
tail -1 $o/tests_m.log
for v in "wg_pair=0,head_onload=0" "wg_pair=0" "wg_pair=1"; do
  UNET_ENGINE="fwd_streams=1,$v" timeout -k 10 400 python tools/layer_times.py --batch 8 --img 128 --dims 3 \
    --out "$o/lt_3d_$v.md" > "$o/lt_3d_$v.log" 2>&1 || { echo "lt 3d rc=$?"; tail -20 "$o/lt_3d_$v.log"; exit 1; }
  head -3 "$o/lt_3d_$v.md" | tail -1
done
for v in 0 2; do
  UNET_ENGINE="fwd_streams=1,wg_pair=$v" timeout -k 10 300 python tools/layer_times.py --batch 1024 --img 128 \
    --out $o/lt_head_p$v.md > $o/lt_head_p$v.log 2>&1 || { echo "lt head rc=$?"; tail -20 $o/lt_head_p$v.log; exit 1; }
  head -3 $o/lt_head_p$v.md | tail -1
done
python tools/lt_diff.py "$o/lt_3d_wg_pair=0,head_onload=0.md" "$o/lt_3d_wg_pair=0.md" 8
python tools/lt_diff.py "$o/lt_3d_wg_pair=0.md" "$o/lt_3d_wg_pair=1.md" 10
python tools/lt_diff.py $o/lt_head_p0.md $o/lt_head_p2.md 14
