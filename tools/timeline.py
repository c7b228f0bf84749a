"""Timeline of one training step from a rocprofv3 --kernel-trace CSV (diagnostics).

usage: python tools/timeline.py <run_results.db|kernel_trace.csv> [marker_substring] [top]

Steps are delimited by the end of the kernel whose name contains the marker (default: the AdamW
kernel, once per step); the last complete step is analysed: its length, the union of busy time over
all streams (the GPU is idle in the rest), each stream's busy time, the time two or more kernels
overlap, and the largest idle gaps with the kernels on either side.
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "adamw"
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    rows = []
    if path.endswith(".db"):  # rocprofv3's default SQLite output
        cur = sqlite3.connect(path).cursor()
        for s, e, n, q in cur.execute("select start, end, name, queue_id from kernels"):
            rows.append((int(s), int(e), n, str(q)))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], q))
    rows.sort()
    ends = [e for s, e, n, q in rows if marker in n]
    if len(ends) < 2:
        sys.exit(f"fewer than two '{marker}' kernels in the trace")
    t0, t1 = ends[-2], ends[-1]
    ks = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    span = t1 - t0
    per = defaultdict(int)
    for s, e, n, q in ks:
        per[q] += e - s
    # union and >= 2-deep overlap by a sweep over start / end events
    ev = sorted([(s, 1) for s, e, n, q in ks] + [(e, -1) for s, e, n, q in ks])
    depth, last, busy, over = 0, t0, 0, 0
    for t, d in ev:
        if depth >= 1:
            busy += t - last
        if depth >= 2:
            over += t - last
        depth += d
        last = t
    # idle gaps: intervals no kernel covers
    gaps = []
    cur_end, prev = t0, None
    for s, e, n, q in ks:
        if s > cur_end:
            gaps.append((s - cur_end, prev, n))
        if e > cur_end:
            cur_end, prev = e, n
    gaps.sort(reverse=True)
    gsum = sum(g for g, _, _ in gaps)
    print(f"step {span / 1e6:.3f} ms, {len(ks)} kernels; busy (any stream) {busy / 1e6:.3f} ms "
          f"({100 * busy / span:.1f}%), >=2 kernels in flight {over / 1e6:.3f} ms, idle {gsum / 1e6:.3f} ms "
          f"in {len(gaps)} gaps")
    for q, t in sorted(per.items(), key=lambda x: -x[1]):
        nq = sum(1 for r in ks if r[3] == q)
        print(f"  queue {q}: {t / 1e6:.3f} ms busy, {nq} kernels")
    hist = defaultdict(lambda: [0, 0])
    for g, _, _ in gaps:
        b = "<2us" if g < 2000 else "2-5us" if g < 5000 else "5-20us" if g < 20000 else ">=20us"
        hist[b][0] += 1
        hist[b][1] += g
    for b in ("<2us", "2-5us", "5-20us", ">=20us"):
        if b in hist:
            print(f"  gaps {b}: {hist[b][0]} totalling {hist[b][1] / 1e6:.3f} ms")
    print(f"largest {top} gaps:")
    for g, a, b in gaps[:top]:
        print(f"  {g / 1e3:8.1f} us  after {str(a)[:60]}  before {b[:60]}")


if __name__ == "__main__":
    main()
