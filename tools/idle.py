"""GPU idle time inside a bench step: wall span of each step's kernels vs their summed durations.
Steps are split at gaps > 200 us (host reset/inject between steps)."""
import csv, sys
path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(path)))
steps, cur = [], [ks[0]]
for a, b in ks[1:]:
    if a - cur[-1][1] > 200_000:
        steps.append(cur); cur = []
    cur.append((a, b))
steps.append(cur)
for s in steps:
    span = (s[-1][1] - s[0][0]) / 1e3
    busy = sum(b - a for a, b in s) / 1e3
    gaps = sorted(((s[i + 1][0] - s[i][1]) / 1e3 for i in range(len(s) - 1)), reverse=True)
    print(f"kernels {len(s):4d} span {span:8.1f} us busy {busy:8.1f} us idle {span - busy:7.1f} us  top gaps {[round(g,1) for g in gaps[:6]]}")
