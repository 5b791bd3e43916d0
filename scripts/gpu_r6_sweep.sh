#!/bin/bash
# Round 6: executor option sweep on the BN / GN fp16 / headline steps (same box, 2 reps each).
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6sweep; mkdir -p $o; : > $o/sweep.txt
b() { timeout -k 10 200 python bench.py --steps 12 --warmup 4 "${@:2}" > $o/b.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/b.log; exit 1; }; echo "$1 $(grep -o '"value": [0-9.]*' $o/b.log)" | tee -a $o/sweep.txt; }
for cfg in "bn:--norm batch" "gn:--norm group --dtype fp16"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  for v in "" "dw_wgs=256" "dw_wgs=1024" "wg_target=384" "wg_target=768" "win_pf=4" "win_pf=16" "dual_stream=0" ""; do
    UNET_ENGINE="$v" b "$tag[$v]" $args
  done
done
for v in "" "dw_wgs=256" "dw_wgs=1024" "win_pf=16" "fwd_offset=4" "fwd_offset=9" ""; do
  UNET_ENGINE="$v" b "head[$v]"
done
