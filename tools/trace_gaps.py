"""Idle time between kernels in a rocprofv3 kernel trace (csv): span, busy time (union of the
kernels' intervals), total idle and the largest gaps, each named by the kernels on either side.
Usage: python tools/trace_gaps.py <kernel_trace.csv> [min_gap_us]"""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"gossip::\(anonymous namespace\)::", "", n).replace("void ", "")
    return re.sub(r"\(.*", "", n)[:40]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
min_gap = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
t0 = int(rows[0]["Start_Timestamp"])
end, busy, gaps = t0, 0, []
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s > end:
        gaps.append(((s - end) / 1e3, short(prev["Kernel_Name"]) if prev else "-", short(r["Kernel_Name"])))
    busy += max(0, e - max(s, end))
    if e > end:
        end, prev = e, r
span = (end - t0) / 1e3
idle = sum(g[0] for g in gaps)
print(f"kernels {len(rows)}, span {span / 1e3:.2f} ms, busy {busy / 1e6:.2f} ms, idle {idle / 1e3:.2f} ms "
      f"in {len(gaps)} gaps")
by = collections.defaultdict(lambda: [0, 0.0])
for g, a, b in gaps:
    if g >= min_gap:
        by[(a, b)][0] += 1
        by[(a, b)][1] += g
for (a, b), (n, t) in sorted(by.items(), key=lambda x: -x[1][1])[:12]:
    print(f"  {n:5d} gaps >= {min_gap:g} us, {t / 1e3:8.2f} ms: {a} -> {b}")
