"""Instruction mix of a kernel's hot loop in a -save-temps .s file (dev tool).
usage: python tools/isa_loop_mix.py file.s kernel_substring"""
import re
import sys
from collections import Counter

path, sub = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sub in l and ":" in l and not l.startswith("\t"))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
body = lines[start:end]
mf = [i for i, l in enumerate(body) if "v_mfma" in l]
# loop = innermost backward branch enclosing the first MFMA
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
best = None
for i, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        n_mf = sum(1 for j in mf if labels[m.group(1)] <= j <= i)
        if n_mf and (best is None or (n_mf, -(i - labels[m.group(1)])) > (best[2], -(best[1] - best[0]))):
            best = (labels[m.group(1)], i, n_mf)
if best is None:
    best = (mf[0], mf[-1], len(mf))
s, e, _ = best
ins = [l.strip().split()[0] for l in body[s:e + 1] if l.strip() and not l.strip().startswith((";", ".")) and not l.startswith(".")]
cat = Counter()
for k in ins:
    if k.startswith("v_mfma"): cat["mfma"] += 1
    elif k.startswith("v_"): cat["valu"] += 1
    elif k.startswith("s_"): cat["salu"] += 1
    elif k.startswith("ds_"): cat["lds"] += 1
    elif k.startswith(("global_", "buffer_")): cat["vmem"] += 1
print(len(ins), dict(cat))
print(Counter(ins).most_common(14))
