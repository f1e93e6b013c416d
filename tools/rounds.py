"""Per-round kernel durations of the last dissemination step in a rocprofv3 kernel trace.

A round starts at bin_emit (dense binned round) or frontier_summary (sparse
frontier round) and ends with round_snapshot; a rebuild or inject before it is
counted with it.
"""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
SHORT = {"bin_count_kernel": "count", "bin_emit_kernel": "emit", "bin_emit_huge_kernel": "emit", "transpose_u16_kernel": "u16", "transpose_u32_kernel": "u32", "bin_serve_kernel": "serve",
         "bin_apply_kernel": "apply", "frontier_summary_kernel": "summ", "frontier_scan_kernel": "scan", "frontier_scan_ns_kernel": "scan_ns",
         "frontier_rebuild_kernel": "rebuild", "frontier_commit_kernel": "commit", "frontier_inject_kernel": "inject", "round_snapshot_kernel": "snap",
         "frontier_bs_emit_kernel": "bs_emit", "frontier_bs_test_kernel": "bs_test"}
STARTS = ("summ", "emit", "rebuild", "bs_emit")


def short(name):
    base = name.replace("(anonymous namespace)::", "").split("(")[0]
    base = base.split("::")[-1]
    return SHORT.get(base.split("<")[0])


rows = list(csv.DictReader(open(path)))
seq = sorted((int(r["Start_Timestamp"]), short(r["Kernel_Name"]),
              (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000) for r in rows)
ks = [x for x in seq if x[1]]
rounds, cur = [], []
for x in ks:
    # (a dense round whose records the previous round's apply emitted starts at its transpose)
    starts = x[1] in STARTS or (x[1] == "u16" and cur and cur[-1][1] == "snap")
    if starts and cur and cur[-1][1] not in ("rebuild", "inject"):
        rounds.append(cur)
        cur = []
    cur.append(x)
if cur:
    rounds.append(cur)
# last step = trailing rounds after the largest gap (the host-side reset/inject between steps)
cut = 0
if len(rounds) > 1:
    gaps = [(rounds[i + 1][0][0] - rounds[i][-1][0], i) for i in range(len(rounds) - 1)]
    cut = max(gaps)[1] + 1
tot = 0
for r in rounds[cut:]:
    t = sum(d for _, _, d in r)
    tot += t
    kind = "sparse" if any(n in ("scan", "scan_ns", "bs_test") for _, n, _ in r) else "dense "
    print(kind, " ".join(f"{n}:{d:6.1f}" for _, n, d in r), f" round {t:6.1f} us")
print(f"rounds {len(rounds) - cut}, kernel time {tot / 1000:.2f} ms")
