"""Per-launch difference of two tools/layer_times.py tables: python tools/lt_diff.py A.md B.md [n]"""
import re
import sys


def load(f):
    d = {}
    for line in open(f):
        m = re.match(r'\| \d+ \| `([^`]+)` \| ([\d.]+) \|', line)
        if m:
            d[m.group(1)] = d.get(m.group(1), 0) + float(m.group(2))
    return d


if __name__ == "__main__":
    a, b = load(sys.argv[1]), load(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    for k in sorted(set(a) | set(b), key=lambda k: -abs(b.get(k, 0) - a.get(k, 0)))[:n]:
        print("%-36s %7.3f %7.3f %+7.3f" % (k, a.get(k, 0), b.get(k, 0), b.get(k, 0) - a.get(k, 0)))
    print("%-36s %7.3f %7.3f %+7.3f" % ("total", sum(a.values()), sum(b.values()), sum(b.values()) - sum(a.values())))
