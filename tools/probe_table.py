"""Aggregate a KDLAE_PROBE_DUMP csv (tag, ms, bytes, flops) per layer tag.

usage: python tools/probe_table.py gpurun_out/probe_c1.csv [...]
"""
import collections
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: [0.0, 0, 0.0, 0.0])
    for r in rows:
        a = agg[r["tag"]]
        a[0] += float(r["ms"])
        a[1] += 1
        a[2] += float(r["bytes"])
        a[3] += float(r["flops"])
    tot = sum(a[0] for a in agg.values())
    print(f"{path}: total {tot:.1f} ms over {len(rows)} launches")
    for k, a in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k:<60} n={a[1]:3d} {a[0]:8.2f}ms {a[0] / a[1] * 1e3:8.1f}us "
              f"{a[2] / a[0] / 1e9:6.2f}TB/s {a[3] / a[0] / 1e9:6.1f}TF/s")
