"""Summary of scripts/gpu_dice_parity.sh runs (gpurun_out/dice/*.jsonl) -> gpurun_out/dice_parity.md.
usage: python scripts/dice_parity_summary.py <seeds...>  (runs of one seed may come from separate GPU calls)"""
import json, statistics, sys
seeds = [int(s) for s in sys.argv[1:]]
import os
runs = [("native bf16, DP=1", "native_dp1"), ("ATen fp32, DP=1", "aten_fp32_dp1"),
        ("native bf16, DP=2 (gloo, 1 card)", "native_dp2"), ("native fp16 + GroupNorm", "native_gn16"),
        ("ATen fp32 + GroupNorm", "aten_gn32"),
        ("native bf16, upsampling decoder, 1 channel", "native_ups"),
        ("ATen fp32, upsampling decoder, 1 channel", "aten_ups")]
# (runs of a path that was not run -- e.g. PAIRS=ups -- are left out)
runs = [r for r in runs if all(os.path.exists("gpurun_out/dice/%s_s%d.jsonl" % (r[1], s)) for s in seeds)]
rows, finals, losses = [], {}, {}
for label, f in runs:
    for seed in seeds:
        recs = [json.loads(l) for l in open("gpurun_out/dice/%s_s%d.jsonl" % (f, seed)) if l.strip()]
        ep = [(r["step"], r["dice"]) for r in recs if r["kind"] == "test"]
        fin = [r for r in recs if r["kind"] == "test_final"][0]
        tr = {r["step"]: r["loss"] for r in recs if r["kind"] == "train"}
        finals.setdefault(f, []).append(fin["dice"])
        losses[(f, seed)] = tr
        rows.append("| %s | %d | %s | %.4f |" % (label, seed, ", ".join("%d: %.4f" % e for e in ep), fin["dice"]))
mean = {k: statistics.mean(v) for k, v in finals.items()}

def loss_gap(a, b):
    out = []
    for seed in seeds:
        la, lb = losses[(a, seed)], losses[(b, seed)]
        steps = sorted(set(la) & set(lb))[-100:]
        out.append(statistics.mean(abs(la[s] - lb[s]) for s in steps) / statistics.mean(lb[s] for s in steps))
    return statistics.mean(out)

# (the header names what was run: the upsampling pair is 1-channel at UPS_LR, default 1e-4)
only_ups = all(f in ("native_ups", "aten_ups") for _, f in runs)
desc = ("upsampling decoder, 128x128x1, global batch 32, lr %s" % os.environ.get("UPS_LR", "1e-4") if only_ups else
        "128x128x4, global batch 32, lr 5e-4; upsampling pair: 1 channel, lr %s" % os.environ.get("UPS_LR", "1e-4"))
out = ["# Dice parity, hard synthetic task (1x MI355X, %s, seeds %s)" % (desc, seeds), "",
       "`scripts/gpu_dice_parity.sh`: per seed the same run (init, data order, dropout streams) through five",
       "paths; test Dice from `Trainer.evaluate` (all full test batches, sharded and allreduced).", "",
       "| run | seed | test Dice per epoch (step: dice) | final test Dice |", "|---|---|---|---|"] + rows
out += ["", "| path | final test Dice per seed | mean |", "|---|---|---|"]
for label, f in runs:
    out.append("| %s | %s | %.4f |" % (label, ", ".join("%.4f" % v for v in finals[f]), mean[f]))
out += ["", "| pair | |seed-mean Dice diff| | bound | mean |loss diff| / loss, last 100 steps | bound | result |",
        "|---|---|---|---|---|---|"]
for la, a, b in (("native bf16 vs ATen fp32", "native_dp1", "aten_fp32_dp1"),
                 ("native DP=1 vs DP=2", "native_dp1", "native_dp2"),
                 ("native fp16+GN vs ATen fp32 GN", "native_gn16", "aten_gn32"),
                 ("upsampling decoder: native bf16 vs ATen fp32", "native_ups", "aten_ups")):
    if a not in mean or b not in mean:
        continue
    d = abs(mean[a] - mean[b])
    g = loss_gap(a, b)
    out.append("| %s | %.4f | 0.02 | %.3f | 0.10 | %s |" % (la, d, g, "pass" if d <= 0.02 and g <= 0.10 else "FAIL"))
open("gpurun_out/dice_parity.md", "w").write("\n".join(out) + "\n")
print("\n".join(out))
