#!/bin/bash
# Round 5: the upsampling decoder at the reference's defaults -- lr 5e-4 (settings_dist.py:19),
# global batch 256 (the reference's per-worker shard, test_dist.py:390), 1 input channel --
# through native bf16, native fp32 (runtime/f32_engine.py) and ATen fp32, 3 seeds.
#   bash scripts/gpu_r5_ups_dice.sh [steps] [seeds...]
set -o pipefail
export TMPDIR=/tmp
# MIOpen's FAST find mode picks naive fp32 NHWC kernels for this decoder (~70 img/s,
# profiles/r5_aten_ups_kernels.md); NORMAL searches once (~3 min, cached for later runs) and
# then runs ~4.7k img/s
export MIOPEN_FIND_MODE=${MIOPEN_FIND_MODE:-NORMAL}
arms=${ARMS:-"native_bf16 native_fp32 aten_fp32"}
steps=${1:-200}; shift || true
seeds=${@:-1 2 3}
o=gpurun_out/dice_ups; mkdir -p $o
COMMON="--synthetic --synthetic_difficulty hard --use_upsampling --in_channels 1 --img_size 128 --batch_size 256 \
  --synthetic_train 2560 --synthetic_test 512 --steps $steps --log_every 1 --no_checkpoint --noexport \
  --noprogress --learning_rate ${LR:-0.0005}"
run() {   # name timeout args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" --log_jsonl $o/$name.jsonl > $o/$name.log 2>&1 \
    || { echo "$name rc=$?"; tail -20 $o/$name.log; exit 1; }
}
for seed in $seeds; do
  [[ $arms == *native_bf16* ]] && run native_bf16_s$seed 300 python train.py $COMMON --seed $seed --backend native --dtype bf16
  [[ $arms == *native_fp32* ]] && run native_fp32_s$seed 400 python train.py $COMMON --seed $seed --backend native --dtype fp32
  [[ $arms == *aten_fp32* ]] && run aten_fp32_s$seed 600 python train.py $COMMON --seed $seed --backend torch --dtype fp32
  echo seed $seed done
done
python scripts/dice_ups_summary.py $o "${LR:-0.0005}" $seeds
