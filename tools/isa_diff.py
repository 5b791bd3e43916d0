"""Instruction-count diff of one kernel between two -S (.s) builds (dev tool).
usage: python tools/isa_diff.py old.s old_kernel_substring new.s new_kernel_substring"""
import sys
from collections import Counter


def body(path, sub):
    lines = open(path).read().split("\n")
    s = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sub in l.split(":")[0] and ":" in l)
    e = next(i for i in range(s, len(lines)) if "s_endpgm" in lines[i])
    return [l.strip().split()[0] for l in lines[s + 1:e]
            if l.startswith("\t") and not l.strip().startswith((";", "."))]


a = Counter(body(sys.argv[1], sys.argv[2]))
b = Counter(body(sys.argv[3], sys.argv[4]))
print("total %d -> %d" % (sum(a.values()), sum(b.values())))
for k in sorted(set(a) | set(b), key=lambda k: -abs(a[k] - b[k])):
    if a[k] != b[k]:
        print("  %-28s %5d %5d" % (k, a[k], b[k]))
