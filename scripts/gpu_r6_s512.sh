#!/bin/bash
# Round 6: 512^2 option A/B (wg_pf=2, win_cp=2) on the current tree.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6s512; mkdir -p $o; : > $o/ab.txt
b() { timeout -k 10 300 python bench.py "${@:2}" > $o/b.log 2>&1 || { echo "bench rc=$?"; tail -20 $o/b.log; exit 1; }; echo "$1 $(grep -o '"value": [0-9.]*' $o/b.log)" | tee -a $o/ab.txt; }
for v in "" "wg_pf=2" "win_cp=2" "wg_pf=2,win_cp=2" ""; do
  UNET_ENGINE="$v" b "s512b64[$v]" --img_size 512 --in_channels 1 --per_gpu_batch 64 --steps 8 --warmup 3
done
for v in "" "wg_pf=2" ""; do
  UNET_ENGINE="$v" b "head[$v]" --steps 20 --warmup 5
done
