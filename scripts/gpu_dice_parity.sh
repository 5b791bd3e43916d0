#!/bin/bash
# Dice parity (BASELINE metric "...; Dice parity"): the same 300-step training run on
# synthetic 128x128x4 BraTS-shaped slices, global batch 32, evaluated every epoch on the
# synthetic test split through Trainer.evaluate, as
#   (a) native HIP executor, bf16, DP=1      (b) ATen (PyTorch) fp32, DP=1
#   (c) native bf16, DP=2 (2 ranks on one card over gloo, 16 per rank)
# for 3 seeds each.  Writes gpurun_out/dice_parity.md (per-epoch test Dice, final, and the
# seed-mean comparison against the 0.02 bound).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/dice
COMMON="--synthetic --in_channels 4 --img_size 128 --batch_size 32 --synthetic_train 1600 --synthetic_test 256 \
  --steps 300 --log_every 50 --no_checkpoint --noexport --noprogress --learning_rate 0.0005"
rm -f gpurun_out/dice/*.jsonl
port=29561
for seed in 1 2 3; do
  timeout -k 10 300 python train.py $COMMON --seed $seed --backend native --dtype bf16 \
    --log_jsonl gpurun_out/dice/native_dp1_s$seed.jsonl > gpurun_out/dice/native_dp1_s$seed.log 2>&1 \
    || { tail -20 gpurun_out/dice/native_dp1_s$seed.log; exit 1; }
  timeout -k 10 400 python train.py $COMMON --seed $seed --backend torch --dtype fp32 \
    --log_jsonl gpurun_out/dice/aten_fp32_dp1_s$seed.jsonl > gpurun_out/dice/aten_fp32_dp1_s$seed.log 2>&1 \
    || { tail -20 gpurun_out/dice/aten_fp32_dp1_s$seed.log; exit 1; }
  port=$((port + 1))
  UNET_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $port train.py $COMMON --seed $seed --backend native --dtype bf16 \
    --log_jsonl gpurun_out/dice/native_dp2_s$seed.jsonl > gpurun_out/dice/native_dp2_s$seed.log 2>&1 \
    || { tail -20 gpurun_out/dice/native_dp2_s$seed.log; exit 1; }
  echo seed $seed done
done
python - <<'PY'
import json, statistics
runs = [("native bf16, DP=1", "native_dp1"), ("ATen fp32, DP=1", "aten_fp32_dp1"),
        ("native bf16, DP=2 (gloo, 1 card)", "native_dp2")]
rows, finals = [], {}
for label, f in runs:
    for seed in (1, 2, 3):
        recs = [json.loads(l) for l in open("gpurun_out/dice/%s_s%d.jsonl" % (f, seed)) if l.strip()]
        ep = [(r["step"], r["dice"]) for r in recs if r["kind"] == "test"]
        fin = [r for r in recs if r["kind"] == "test_final"][0]
        tr = [(r["step"], r["loss"]) for r in recs if r["kind"] == "train"]
        finals.setdefault(f, []).append(fin["dice"])
        rows.append("| %s | %d | %s | %.4f | %s |" % (label, seed, ", ".join("%d: %.4f" % e for e in ep), fin["dice"],
                                                   ", ".join("%d: %.3f" % t for t in tr)))
mean = {k: statistics.mean(v) for k, v in finals.items()}
out = ["# Dice parity (1x MI355X, synthetic 128x128x4, global batch 32, 300 steps, lr 5e-4, 3 seeds)", "",
       "`scripts/gpu_dice_parity.sh`: per seed the same run (init, data order, dropout streams) through",
       "three paths; test Dice from `Trainer.evaluate` (all full test batches, sharded and allreduced).", "",
       "| run | seed | test Dice per epoch (step: dice) | final test Dice | train loss (step: loss) |",
       "|---|---|---|---|---|"] + rows
out += ["", "| path | final test Dice (seeds 1, 2, 3) | mean |", "|---|---|---|"]
for label, f in runs:
    out.append("| %s | %s | %.4f |" % (label, ", ".join("%.4f" % v for v in finals[f]), mean[f]))
d1 = abs(mean["native_dp1"] - mean["aten_fp32_dp1"])
d2 = abs(mean["native_dp1"] - mean["native_dp2"])
out += ["", "| check (seed means) | abs diff | bound | result |", "|---|---|---|---|",
        "| native bf16 vs ATen fp32 (DP=1) | %.4f | 0.02 | %s |" % (d1, "pass" if d1 <= 0.02 else "FAIL"),
        "| native DP=1 vs DP=2 | %.4f | 0.02 | %s |" % (d2, "pass" if d2 <= 0.02 else "FAIL")]
open("gpurun_out/dice_parity.md", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
