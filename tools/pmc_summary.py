"""Per-kernel PMC summary from a rocprofv3 ``--pmc`` sqlite output (rocpd schema):
counter values summed over instances per dispatch, averaged over dispatches.

    python tools/pmc_summary.py gpurun_out/pmc1/pmc_results.db [kernel-substring]
"""
import sqlite3
import sys


def summary(db, needle=""):
    con = sqlite3.connect(db)
    q = """select s.display_name, d.id, (d."end" - d.start), i.name, sum(e.value)
           from rocpd_pmc_event e
           join rocpd_info_pmc i on e.pmc_id = i.id
           join rocpd_kernel_dispatch d on d.event_id = e.event_id
           join rocpd_info_kernel_symbol s on s.id = d.kernel_id
           group by d.id, i.name"""
    out = {}
    for kname, did, dur, cname, val in con.execute(q):
        if needle and needle not in kname:
            continue
        k = out.setdefault(kname, {"_d": set(), "_t": 0.0})
        if did not in k["_d"]:
            k["_d"].add(did)
            k["_t"] += dur
        k[cname] = k.get(cname, 0.0) + val
    res = {}
    for kname, k in out.items():
        n = len(k["_d"])
        res[kname] = dict({c: v / n for c, v in k.items() if not c.startswith("_")},
                          dispatches=n, avg_ns=k["_t"] / n)
    return res


if __name__ == "__main__":
    r = summary(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
    for k, v in r.items():
        print(k[:100])
        for c, x in sorted(v.items()):
            print("   %-28s %.4g" % (c, x))
