"""Summarise rocprofv3 --pmc CSVs (one counter group per pass) per kernel.

FETCH_SIZE/WRITE_SIZE are in KiB; per MI355X_MICROARCH.md §HBM the gfx950
FETCH_SIZE reads half the bytes of a wide streaming read, so the corrected read
traffic is 2 x FETCH_SIZE (reported as both).  Usage:
    python tools/pmc_summary.py gpurun_out/pmc [--json out.json]
"""
import collections
import csv
import glob
import json
import os
import sys


def kname(s):
    s = s.replace("(anonymous namespace)::", "")
    return s.split("(")[0].split("::")[-1]


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            per[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    d = sys.argv[1]
    per = load(d)
    out = {}
    for k, cs in sorted(per.items()):
        row = {c: sum(v) / len(v) for c, v in cs.items()}
        row["dispatches"] = max(len(v) for v in cs.values())
        if "FETCH_SIZE" in row:
            row["read_MB_raw"] = row["FETCH_SIZE"] * 1024 / 1e6
            row["read_MB_corrected"] = 2 * row["read_MB_raw"]
        if "WRITE_SIZE" in row:
            row["write_MB"] = row["WRITE_SIZE"] * 1024 / 1e6
        if "TCC_HIT_sum" in row:
            row["l2_hit"] = row["TCC_HIT_sum"] / max(1.0, row["TCC_HIT_sum"] + row["TCC_MISS_sum"])
        out[k] = row
        print(k, {a: round(b, 3) for a, b in row.items()})
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
