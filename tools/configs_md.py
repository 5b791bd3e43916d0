"""profiles/r5_configs.md from a configs.jsonl of scripts/gpu_r5_configs.sh.
usage: python tools/configs_md.py <configs.jsonl> <out.md>"""
import json
import sys

src, out = sys.argv[1], sys.argv[2]
rows = [json.loads(l) for l in open(src) if l.strip()]
L = ["# Every BASELINE config (1x MI355X, `scripts/gpu_r<N>_configs.sh`)", "",
     "One `bench.py` line per config (full training step: forward, loss, backward, TF-Adam; synthetic data, "
     "random init). TF/s = img/s x the step's conv / transposed-conv FLOPs per image (`tools/config_flops.py`, "
     "3 x forward MACs x 2).", "",
     "| tag | model | dtype | per-GPU batch | img/s | ms/step | GFLOP/img | TF/s | args |",
     "|---|---|---|---|---|---|---|---|---|"]
for r in rows:
    c = r.get("config", {})
    L.append("| %s | %s | %s | %s | %.1f | %.2f | %s | %s | `%s` |" % (
        r.get("tag"), c.get("model", "").split(" (")[0], r.get("dtype"), c.get("global_batch"), r["value"],
        r["ms_per_step"], r.get("gflop_per_img"), r.get("tflops"), r.get("args", "")))
open(out, "w").write("\n".join(L) + "\n")
print("\n".join(L))
