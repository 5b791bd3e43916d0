"""Summary of scripts/gpu_r5_ups_dice.sh (upsampling decoder, 1 channel, global batch 256).
usage: python scripts/dice_ups_summary.py <dir> <lr> <seeds...>  -> <dir>/summary.md"""
import json
import statistics
import sys

d, lr, seeds = sys.argv[1], sys.argv[2], [int(s) for s in sys.argv[3:]]
arms = [("native bf16", "native_bf16"), ("native fp32", "native_fp32"), ("ATen fp32", "aten_fp32")]
rows, finals, losses, steps_run, collapse = [], {}, {}, {}, {}
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
        steps_run[(f, s)] = max(tr) if tr else 0
        # collapse: the loss jumps to the all-background plateau (log(St + 1) ~ 10.8) and stays
        jump = next((k for k in sorted(tr) if tr[k] > 9.0), None)
        collapse[(f, s)] = (jump, fin < 0.01)
        first = ", ".join("%.4f" % tr[k] for k in sorted(tr)[:8])
        rows.append("| %s | %d | %d | %s | %s | %.4f |" % (label, s, steps_run[(f, s)], first,
                                                        ", ".join("%d: %.3f" % e for e in ep[::4]), fin))
out = ["# Upsampling decoder at the reference's defaults (1x MI355X, 128x128x1 hard synthetic task, "
       "global batch 256, lr %s, seeds %s)" % (lr, seeds), "",
       "`scripts/gpu_r5_ups_dice.sh`: per seed the same run (init, data order, dropout streams) through native "
       "bf16, native fp32 (`runtime/f32_engine.py`) and ATen fp32 (MIOpen, `MIOPEN_FIND_MODE=NORMAL`); test Dice "
       "from `Trainer.evaluate` every 10 steps. The reference's defaults: lr 5e-4 (`settings_dist.py:19`), "
       "256 images per worker (`test_dist.py:390`), `--use_upsampling` (`test_dist.py:84-85`).", "",
       "| run | seed | steps | training loss, steps 1-8 | test Dice (step: dice) | final test Dice |",
       "|---|---|---|---|---|---|"] + rows
out += ["", "## Outcome per seed", "",
        "| seed | " + " | ".join(l for l, _ in arms) + " |", "|---|" + "---|" * len(arms)]
for s in seeds:
    cells = []
    for _, f in arms:
        if (f, s) not in collapse:
            cells.append("-")
            continue
        jump, dead = collapse[(f, s)]
        cells.append(("collapsed at step %d" % jump) if dead and jump else
                     ("escaped (loss spike at step %d), final Dice %.3f" % (jump, finals[f][s]) if jump else
                      "trained, final Dice %.3f" % finals[f][s]))
    out.append("| %d | %s |" % (s, " | ".join(cells)))
out += ["", "| arm | final test Dice per seed | seed mean |", "|---|---|---|"]
for label, f in arms:
    if f in finals:
        v = [finals[f][s] for s in seeds if s in finals[f]]
        out.append("| %s | %s | %.4f |" % (label, ", ".join("%.4f" % x for x in v), statistics.mean(v)))
out += ["", "| pair | per-seed |Dice diff| | seed-mean |diff| | bound | early-loss max rel diff (steps 1-8) |",
        "|---|---|---|---|---|"]
for la, a, b in (("native bf16 vs ATen fp32", "native_bf16", "aten_fp32"),
                 ("native fp32 vs ATen fp32", "native_fp32", "aten_fp32"),
                 ("native bf16 vs native fp32", "native_bf16", "native_fp32")):
    if a not in finals or b not in finals:
        continue
    common = [s for s in seeds if s in finals[a] and s in finals[b]]
    ps = [abs(finals[a][s] - finals[b][s]) for s in common]
    mm = abs(statistics.mean(finals[a][s] for s in common) - statistics.mean(finals[b][s] for s in common))
    el = max(abs(losses[(a, s)][k] - losses[(b, s)][k]) / abs(losses[(b, s)][k])
             for s in common for k in range(1, 9) if k in losses[(a, s)] and k in losses[(b, s)])
    out.append("| %s | %s | %.4f | 0.02 | %.2e |" % (la, ", ".join("%.4f" % x for x in ps), mm, el))
open("%s/summary.md" % d, "w").write("\n".join(out) + "\n")
print("\n".join(out))
