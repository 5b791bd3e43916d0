#!/bin/bash
# Round 6: 3D b8 confirmation A/B of the sweep's best options (interleaved, 3 reps).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6sweep3d; mkdir -p $o; : > $o/sweep_b.txt
b() { timeout -k 10 200 python bench.py --dims 3 --steps 6 --warmup 2 "${@:2}" > $o/b.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/b.log; exit 1; }; echo "$1 $(grep -o '"value": [0-9.]*' $o/b.log)" | tee -a $o/sweep_b.txt; }
for r in 1 2 3; do
  for v in "" "fwd_streams=1" "fwd_offset=3" "fwd_streams=1,wg_target=1024"; do
    UNET_ENGINE="$v" b "d3[$v]"
  done
done
b "d3_b16[]" --per_gpu_batch 16
UNET_ENGINE="fwd_streams=1" b "d3_b16[fwd_streams=1]" --per_gpu_batch 16
