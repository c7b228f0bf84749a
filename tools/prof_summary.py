"""Summarise a rocprofv3 kernel-trace database (.db) or CSV: per-kernel totals, count, average.

usage: python tools/prof_summary.py <run_results.db|kernel_trace.csv> [--per N] [--by-grid]
"""
import argparse
import collections
import csv
import re
import sqlite3


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = n.replace("void ", "").replace("kdlae::", "")
    return n


def rows_from(path):
    if path.endswith(".db"):
        cur = sqlite3.connect(path).cursor()
        q = "select name, duration, grid_x, grid_y, grid_z, workgroup_x, lds_size, vgpr_count, accum_vgpr_count from kernels"
        for r in cur.execute(q):
            yield dict(name=r[0], dur=r[1], grid=(r[2], r[3], r[4]), wg=r[5], lds=r[6], vgpr=r[7], agpr=r[8])
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                yield dict(name=r["Kernel_Name"], dur=int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                           grid=(r.get("Grid_Size_X"), r.get("Grid_Size_Y"), r.get("Grid_Size_Z")),
                           wg=r.get("Workgroup_Size_X"), lds=r.get("LDS_Block_Size"), vgpr=r.get("VGPR_Count"),
                           agpr=r.get("Accum_VGPR_Count"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--per", type=float, default=1.0, help="divide totals by this (e.g. forwards)")
    ap.add_argument("--by-grid", action="store_true")
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: [0, 0])
    for r in rows_from(a.path):
        key = short(r["name"]) + (f" grid={r['grid']}" if a.by_grid else "")
        tot[key][0] += r["dur"]
        tot[key][1] += 1
    all_ns = sum(v[0] for v in tot.values())
    print(f"{'kernel':<70} {'ms/per':>10} {'%':>6} {'count/per':>10} {'avg us':>9}")
    for k, (ns, n) in sorted(tot.items(), key=lambda kv: -kv[1][0]):
        print(f"{k[:70]:<70} {ns / 1e6 / a.per:>10.3f} {100 * ns / all_ns:>6.2f} {n / a.per:>10.1f} {ns / n / 1e3:>9.1f}")
    print(f"{'TOTAL':<70} {all_ns / 1e6 / a.per:>10.3f}")


if __name__ == "__main__":
    main()
