"""Markdown table of the SQ wave-cycle breakdown per kernel from a ``gpu_stall_pmc.sh`` run:
share of wave-cycles parked on s_waitcnt / barriers (SQ_WAIT_ANY), stalled on issue
(SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY), plus MFMA busy as a fraction of the
kernel's SIMD-cycles (SQ_VALU_MFMA_BUSY_CYCLES / (time x clock x SIMDs)).

    python tools/stall_table.py gpurun_out/stall_r3/pmc1/run_results.db [--clock-ghz 2.4] [--simds 1024]
"""
import argparse
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summary  # noqa: E402


def short(name):
    """Readable kernel name: the function name plus its leading template arguments."""
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(\w+)<([^<>]*)", name)
    if m:
        return "%s<%s>" % (m.group(1).split("::")[-1], m.group(2)[:40])
    return name.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--clock-ghz", type=float, default=2.4)
    ap.add_argument("--simds", type=int, default=1024)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = []
    for k, v in summary(a.db).items():
        tot_ms = v["avg_ns"] * v["dispatches"] / 1e6
        wc = v.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        simd_cycles = v["avg_ns"] * a.clock_ghz * a.simds
        rows.append((tot_ms, short(k), v["dispatches"], v["avg_ns"] / 1e3, v.get("SQ_WAIT_ANY", 0) / wc,
                     v.get("SQ_WAIT_INST_ANY", 0) / wc, v.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                     v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / simd_cycles))
    rows.sort(reverse=True)
    total = sum(r[0] for r in rows)
    print("| kernel | launches | avg us | total ms | % | wait (waitcnt/barrier) | issue-stall | issuing | MFMA busy |")
    print("|---|---|---|---|---|---|---|---|---|")
    for r in rows[:a.top]:
        print("| `%s` | %d | %.1f | %.3f | %.1f | %.2f | %.2f | %.2f | %.2f |"
              % (r[1], r[2], r[3], r[0], 100 * r[0] / total, r[4], r[5], r[6], r[7]))


if __name__ == "__main__":
    main()
