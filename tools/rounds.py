"""Per-round kernel durations of the last dissemination step in a rocprofv3 kernel trace."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
names = ("bin_emit_kernel", "transpose_u16_kernel", "bin_serve_kernel", "bin_apply_kernel")
rows = list(csv.DictReader(open(path)))
seq = sorted((int(r["Start_Timestamp"]),
              r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1].split("<")[0],
              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000) for r in rows)
ks = [x for x in seq if x[1] in names]
starts = [i for i, x in enumerate(ks) if x[1] == names[0]]
rounds = [ks[a:b] for a, b in zip(starts, starts[1:] + [len(ks)])]
# last step = trailing rounds after the largest gap between consecutive emits
gaps = [(rounds[i + 1][0][0] - rounds[i][-1][0], i) for i in range(len(rounds) - 1)]
cut = max(gaps)[1] + 1 if gaps else 0
tot = 0
for r in rounds[cut:]:
    t = sum(d for _, _, d in r)
    tot += t
    print(" ".join(f"{n.split('_')[1][:6]}:{d:6.1f}" for _, n, d in r), f" round {t:6.1f} us")
print(f"rounds {len(rounds) - cut}, kernel time {tot / 1000:.2f} ms")
