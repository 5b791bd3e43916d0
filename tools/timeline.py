"""Step timeline from a rocprofv3 --kernel-trace run: where the wall time of ONE
training step goes (forward / backward spans, per-queue busy time, overlap of the
dual-stream backward, idle gaps between kernels).

usage: python tools/timeline.py <kernel_trace.csv> [title]

A step ends with the fused Adam launch (adam_pack_kernel); the last complete step
of the trace is analysed.  The forward ends at the head's loss kernel
(head_finish / head_fwd)."""
import csv
import sys


def short(n):
    i = n.find("kernel<")
    if i >= 0:
        return n[n.rfind("::", 0, i) + 2: n.find(">", i) + 1]
    return n.replace("unet::(anonymous namespace)::", "").split("(")[0][:60]


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e in iv:
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            tot += cur_e - cur_s
            gaps.append((cur_e, s))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot, gaps


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    rows = list(csv.DictReader(open(path)))
    qk = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)
    ks = []
    for r in rows:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                   r.get(qk, "0") if qk else "0"))
    ks.sort()
    ends = [i for i, k in enumerate(ks) if "adam_pack" in k[2]]
    if len(ends) < 2:
        print("need two adam_pack launches in the trace")
        return
    step = ks[ends[-2] + 1: ends[-1] + 1]
    t0 = step[0][0]
    t1 = max(k[1] for k in step)
    fwd_end = next((k[1] for k in step if k[2].startswith(("head_finish", "head_fwd")) or "norm_head_loss" in k[2]),
                   None)
    span = (t1 - t0) / 1e6
    busy, gaps = union([(k[0], k[1]) for k in step])
    ksum = sum(k[1] - k[0] for k in step) / 1e6
    print("# %s\n" % title)
    print("| quantity | ms |")
    print("|---|---|")
    print("| step span (first kernel start -> last kernel end) | %.3f |" % span)
    if fwd_end:
        fb, _ = union([(k[0], min(k[1], fwd_end)) for k in step if k[0] < fwd_end])
        print("| forward span | %.3f |" % ((fwd_end - t0) / 1e6))
        print("| forward kernel-busy | %.3f |" % (fb / 1e6))
        bb, _ = union([(max(k[0], fwd_end), k[1]) for k in step if k[1] > fwd_end])
        print("| backward + optimizer span | %.3f |" % ((t1 - fwd_end) / 1e6))
        print("| backward + optimizer kernel-busy (union) | %.3f |" % (bb / 1e6))
    print("| any-kernel-busy (union) | %.3f |" % (busy / 1e6))
    print("| idle (no kernel running) | %.3f |" % ((t1 - t0 - busy) / 1e6))
    print("| sum of kernel durations | %.3f |" % ksum)
    print("| overlap gain (sum - union) | %.3f |" % (ksum - busy / 1e6))
    print("| launches | %d |" % len(step))
    queues = sorted({k[3] for k in step})
    print("\n| queue | launches | kernel ms |")
    print("|---|---|---|")
    for q in queues:
        qs = [k for k in step if k[3] == q]
        print("| %s | %d | %.3f |" % (q, len(qs), sum(k[1] - k[0] for k in qs) / 1e6))
    big = sorted(gaps, key=lambda g: g[0] - g[1])[:10]
    if big:
        print("\nlargest idle gaps (us, after kernel):")
        for s, e in big:
            prev = max((k for k in step if k[1] <= s), key=lambda k: k[1])
            print("- %.1f after `%s`" % ((e - s) / 1e3, prev[2]))
    print("\n| start us | dur us | queue | kernel |")
    print("|---|---|---|---|")
    for k in step:
        print("| %.1f | %.1f | %s | `%s` |" % ((k[0] - t0) / 1e3, (k[1] - k[0]) / 1e3, k[3], k[2]))


if __name__ == "__main__":
    main()
