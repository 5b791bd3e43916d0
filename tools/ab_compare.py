"""Compare per-launch layer_times tables of two builds (min over repeated runs).
usage: python tools/ab_compare.py base1.md [base2.md ...] -- new1.md [new2.md ...]"""
import re
import sys


def load(paths):
    best = {}
    for f in paths:
        for line in open(f):
            m = re.match(r"\| \d+ \| `([^`]+)` \| ([\d.]+) \|", line)
            if m:
                k, v = m.group(1), float(m.group(2))
                best[k] = min(best.get(k, 1e9), v)
    return best


args = sys.argv[1:]
i = args.index("--")
a, b = load(args[:i]), load(args[i + 1:])
ta, tb = sum(a.values()), sum(b.values())
print("# A/B per-launch times (min over runs): base %.3f ms, new %.3f ms (%+.1f %%)\n" % (ta, tb, 100 * (tb / ta - 1)))
print("| launch | base ms | new ms | change |")
print("|---|---|---|---|")
for k in a:
    if k in b:
        print("| `%s` | %.4f | %.4f | %+.1f %% |" % (k, a[k], b[k], 100 * (b[k] / a[k] - 1)))
