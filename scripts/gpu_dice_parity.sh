#!/bin/bash
# Dice parity (BASELINE metric "...; Dice parity") in a regime where it discriminates:
# the same training run on synthetic 128x128x4 BraTS-shaped slices of the HARD synthetic
# task (datasets.synthetic_brats difficulty="hard": small low-contrast lesions, Dice
# plateau well below 1), global batch 32, evaluated every epoch through Trainer.evaluate:
#   (a) native HIP, bf16, DP=1           (b) ATen (PyTorch) fp32, DP=1
#   (c) native bf16, DP=2 (2 ranks, gloo on one card, 16 per rank)
#   (d) native fp16 + GroupNorm, DP=1    (e) ATen fp32 + GroupNorm, DP=1
#   (f) native bf16, upsampling decoder, 1 input channel   (g) the same on ATen fp32
# for the seeds given (default 1 2 3).  PAIRS="ups" runs only (f) / (g).  Writes gpurun_out/dice_parity.md: per-epoch test Dice,
# final Dice, seed means against the 0.02 bound, and the mean |delta| of the per-step
# training loss over the last 100 steps relative to the loss.
#   bash scripts/gpu_dice_parity.sh [steps] [seeds...]
set -o pipefail
export TMPDIR=/tmp
# (the ATen fp32 arms: immediate-mode MIOpen kernel choice, no per-shape search)
export MIOPEN_FIND_MODE=${MIOPEN_FIND_MODE:-FAST}
steps=${1:-300}; shift || true
seeds=${@:-1 2 3}
mkdir -p gpurun_out/dice
COMMON="--synthetic --synthetic_difficulty hard --in_channels 4 --img_size 128 --batch_size 32 \
  --synthetic_train 1600 --synthetic_test 256 --steps $steps --log_every 1 --no_checkpoint --noexport \
  --noprogress --learning_rate 0.0005"
port=29561
run() {   # name timeout args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" --log_jsonl gpurun_out/dice/$name.jsonl > gpurun_out/dice/$name.log 2>&1 \
    || { tail -20 gpurun_out/dice/$name.log; exit 1; }
}
# (UPS_LR: the 1-channel upsampling decoder jumps into the all-background saturation at step 3 at
# lr 5e-4 on both backends -- whether a run escapes it depends on rounding -- so its pair runs at
# UPS_LR, default 1e-4)
UPS="--use_upsampling --in_channels 1 --learning_rate ${UPS_LR:-0.0001}"
for seed in $seeds; do
  run native_ups_s$seed 300 python train.py $COMMON $UPS --seed $seed --backend native --dtype bf16
  run aten_ups_s$seed 500 python train.py $COMMON $UPS --seed $seed --backend torch --dtype fp32
  if [ "${PAIRS:-all}" = ups ]; then echo seed $seed done; continue; fi
  run native_dp1_s$seed 300 python train.py $COMMON --seed $seed --backend native --dtype bf16
  run aten_fp32_dp1_s$seed 500 python train.py $COMMON --seed $seed --backend torch --dtype fp32
  port=$((port + 1))
  UNET_DIST_BACKEND=gloo run native_dp2_s$seed 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $port train.py $COMMON --seed $seed --backend native --dtype bf16
  run native_gn16_s$seed 300 python train.py $COMMON --seed $seed --backend native --dtype fp16 --norm group
  run aten_gn32_s$seed 500 python train.py $COMMON --seed $seed --backend torch --dtype fp32 --norm group
  echo seed $seed done
done
python scripts/dice_parity_summary.py $seeds
