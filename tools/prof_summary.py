"""Summarise a rocprofv3 --kernel-trace --stats run into a markdown table.
usage: python tools/prof_summary.py <prof_dir> <steps_profiled> [title]"""
import csv
import os
import sys

d, steps = sys.argv[1], int(sys.argv[2])
title = sys.argv[3] if len(sys.argv) > 3 else d
rows = list(csv.DictReader(open(os.path.join(d, "prof_kernel_stats.csv"))))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("# %s\n" % title)
print("GPU kernel time per profiled step: %.2f ms (%d steps incl. warmup)\n" % (tot / steps / 1e6, steps))
print("| kernel | calls/step | ms/step | % |")
print("|---|---|---|---|")
for r in rows:
    n = r["Name"]
    i = n.find("kernel<")
    if i >= 0:
        n = n[n.rfind("::", 0, i) + 2: n.find(">", i) + 1]
    else:
        n = n.replace("unet::(anonymous namespace)::", "").split("(")[0][:70]
    pct = 100 * float(r["TotalDurationNs"]) / tot
    if pct < 0.1:
        continue
    print("| `%s` | %.1f | %.3f | %.1f |" % (n, int(r["Calls"]) / steps, float(r["TotalDurationNs"]) / steps / 1e6, pct))
