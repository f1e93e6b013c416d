"""Sparse-round scan / commit times (us) of the last step in a rocprofv3 kernel trace, in round
order, plus their sum (dense rounds shown as D).  Usage: sparse_rounds.py <kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
seq = []
for r in rows:
    n, d = r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "frontier_scan" in n:
        seq.append(["S", d, 0.0])
    elif "frontier_commit" in n and seq:
        seq[-1][2] = d
    elif "bin_emit" in n:
        seq.append(["D", 0.0, 0.0])
# the last step: from the last inject-like start (a sparse round after a dense run that follows)
last = len(seq)
for i in range(len(seq) - 1, 0, -1):
    if seq[i][0] == "D" and seq[i - 1][0] == "S" and i < last - 2:
        break
step = seq[-16:]
print(" ".join(f"{k}:{a:.0f}+{b:.0f}" if k == "S" else "D" for k, a, b in step))
print(f"sparse scan sum {sum(a for k, a, b in step if k == 'S'):.0f} us, commit sum {sum(b for k, a, b in step if k == 'S'):.0f} us")
