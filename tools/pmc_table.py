"""Merge the PMC passes of scripts/gpu_profile.sh into one markdown table.

    python tools/pmc_table.py gpurun_out/prof_<tag>

Per kernel (averaged over dispatches): duration, MFMA utilisation
(SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x duration x 2.4 GHz; counter passes run
at lower clocks, so a lower bound), VALU instructions per MFMA, LDS bank-conflict
share, HBM-side bytes (FETCH_SIZE doubled: on gfx950 it reports half the bytes of a
wide streaming read, MI355X_MICROARCH.md 'HBM') and the implied bandwidth.
"""
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summary  # noqa: E402


def _short(n):
    i = n.find("kernel<")
    if i >= 0:
        return n[n.rfind("::", 0, i) + 2 if "::" in n[:i] else 0: n.find(">", i) + 1].replace("void ", "")
    return n.replace("unet::(anonymous namespace)::", "").split("(")[0][:60]


def main(d):
    merged = {}
    for p in sorted(glob.glob(os.path.join(d, "pmc*"))):
        dbs = glob.glob(os.path.join(p, "**", "*.db"), recursive=True)
        if not dbs:
            continue
        for k, v in summary(dbs[0]).items():
            m = merged.setdefault(k, {})
            for c, x in v.items():
                if c in ("dispatches", "avg_ns"):
                    m.setdefault(c, x)
                else:
                    m[c] = x
    rows = []
    for k, m in merged.items():
        ns = m.get("avg_ns", 0.0)
        if ns <= 0:
            continue
        mf = m.get("SQ_VALU_MFMA_BUSY_CYCLES")
        util = 100.0 * mf / (1024 * ns * 2.4) if mf is not None else None
        vm = (m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"]) if m.get("SQ_INSTS_MFMA") else None
        lds = (100.0 * m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]) if m.get("SQ_LDS_IDX_ACTIVE") else None
        fb = 2 * 1024 * m["FETCH_SIZE"] if "FETCH_SIZE" in m else None    # FETCH_SIZE is in KiB
        wb = 1024 * m["WRITE_SIZE"] if "WRITE_SIZE" in m else None
        bw = ((fb or 0) + (wb or 0)) / ns if (fb is not None or wb is not None) else None  # B/ns = GB/s
        rows.append((ns * m.get("dispatches", 1), k, ns, util, vm, lds, fb, wb, bw, m.get("dispatches", 0)))
    rows.sort(reverse=True)
    f = lambda x, fmt: "" if x is None else fmt % x   # noqa: E731
    print("| kernel | dispatches | avg us | MFMA util % | VALU/MFMA | LDS conflict % | read MB | write MB | TB/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    for _, k, ns, util, vm, lds, fb, wb, bw, n in rows[:40]:
        print("| `%s` | %d | %.1f | %s | %s | %s | %s | %s | %s |" % (
            _short(k), n, ns / 1e3, f(util, "%.1f"), f(vm, "%.1f"), f(lds, "%.1f"),
            f(fb and fb / 1e6, "%.0f"), f(wb and wb / 1e6, "%.0f"), f(bw and bw / 1e3, "%.2f")))


if __name__ == "__main__":
    main(sys.argv[1])
