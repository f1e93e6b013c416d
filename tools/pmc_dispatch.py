"""Per-dispatch counters of one kernel from rocprofv3 --pmc CSVs (all passes in a directory).
Usage: python tools/pmc_dispatch.py DIR KERNEL_SUBSTRING"""
import collections, csv, glob, os, sys

d, pat = sys.argv[1], sys.argv[2]
per_pass = {}
for f in sorted(glob.glob(os.path.join(d, "*_counter_collection.csv"))):
    rows = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        rows.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    per_pass[f] = list(rows.values())
n = max((len(v) for v in per_pass.values()), default=0)
for i in range(n):
    row = {}
    for v in per_pass.values():
        if i < len(v):
            row.update(v[i])
    print(i, " ".join(f"{k}={v:.3g}" for k, v in sorted(row.items())))
