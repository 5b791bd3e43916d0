#!/bin/bash
# Round 6: executor option sweep on the 3D b8 step (same box).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6sweep3d; mkdir -p $o; : > $o/sweep.txt
b() { timeout -k 10 200 python bench.py --dims 3 --steps 6 --warmup 2 "${@:2}" > $o/b.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/b.log; exit 1; }; echo "$1 $(grep -o '"value": [0-9.]*' $o/b.log)" | tee -a $o/sweep.txt; }
for v in "" "wg_target=256" "wg_target=384" "wg_target=768" "wg_target=1024" "fwd_offset=3" "fwd_offset=9" "fwd_streams=1" "dual_stream=0" "wg_pair=1" ""; do
  UNET_ENGINE="$v" b "d3[$v]"
done
