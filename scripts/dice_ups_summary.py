"""Summary of scripts/gpu_r5_ups_dice.sh (upsampling decoder, 1 channel, global batch 256).
usage: python scripts/dice_ups_summary.py <dir> <lr> <seeds...>  -> <dir>/summary.md"""
import json
import statistics
import sys

d, lr, seeds = sys.argv[1], sys.argv[2], [int(s) for s in sys.argv[3:]]
arms = [("native bf16", "native_bf16"), ("native fp32", "native_fp32"), ("ATen fp32", "aten_fp32")]
rows, finals, losses = [], {}, {}
for label, f in arms:
    for s in seeds:
        try:
            recs = [json.loads(l) for l in open("%s/%s_s%d.jsonl" % (d, f, s)) if l.strip()]
        except OSError:
            continue
        tr = {r["step"]: r["loss"] for r in recs if r["kind"] == "train"}
        ep = [(r["step"], r["dice"]) for r in recs if r["kind"] == "test"]
        fr = [r for r in recs if r["kind"] == "test_final"] or [r for r in recs if r["kind"] == "test"][-1:]
        fin = fr[0]["dice"]
        finals.setdefault(f, {})[s] = fin
        losses[(f, s)] = tr
        first = ", ".join("%.4f" % tr[k] for k in sorted(tr)[:8])
        rows.append("| %s | %d | %s | %s | %.4f |" % (label, s, first,
                                                     ", ".join("%d: %.3f" % e for e in ep[::3]), fin))
out = ["# Upsampling decoder at the reference's defaults (1x MI355X, 128x128x1 hard synthetic task, "
       "global batch 256, lr %s, seeds %s)" % (lr, seeds), "",
       "`scripts/gpu_r5_ups_dice.sh`: per seed the same run (init, data order, dropout streams) through native "
       "bf16, native fp32 (runtime/f32_engine.py) and ATen fp32; test Dice from `Trainer.evaluate`.", "",
       "| run | seed | training loss, steps 1-8 | test Dice (every 3rd epoch) | final test Dice |",
       "|---|---|---|---|---|"] + rows
out += ["", "| arm | final test Dice per seed | mean |", "|---|---|---|"]
for label, f in arms:
    if f in finals:
        v = [finals[f][s] for s in seeds if s in finals[f]]
        out.append("| %s | %s | %.4f |" % (label, ", ".join("%.4f" % x for x in v), statistics.mean(v)))
out += ["", "| pair | per-seed |Dice diff| | seed-mean |diff| | bound | early-loss max rel diff (steps 1-8) |",
        "|---|---|---|---|---|"]
for la, a, b in (("native bf16 vs ATen fp32", "native_bf16", "aten_fp32"),
                 ("native fp32 vs ATen fp32", "native_fp32", "aten_fp32")):
    if a not in finals or b not in finals:
        continue
    ps = [abs(finals[a][s] - finals[b][s]) for s in seeds if s in finals[a] and s in finals[b]]
    mm = abs(statistics.mean(finals[a].values()) - statistics.mean(finals[b].values()))
    el = max(abs(losses[(a, s)][k] - losses[(b, s)][k]) / abs(losses[(b, s)][k])
             for s in seeds for k in range(1, 9) if (a, s) in losses and k in losses[(a, s)])
    out.append("| %s | %s | %.4f | 0.02 | %.2e |" % (la, ", ".join("%.4f" % x for x in ps), mm, el))
open("%s/summary.md" % d, "w").write("\n".join(out) + "\n")
print("\n".join(out))
