"""Summarize rocprofv3 --stats kernel tables: name (short), calls, average us.
Usage: kstats.py <run_kernel_stats.csv> [substring filter ...]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
keys = sys.argv[2:]
for r in rows:
    n = r["Name"]
    if keys and not any(k in n for k in keys):
        continue
    n = re.sub(r"gossip::\(anonymous namespace\)::", "", n).replace("void ", "")
    n = re.sub(r"\(gossip::.*", "", n)[:44]
    print(f"  {n:44s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e3:8.1f} us "
          f"total {float(r['TotalDurationNs']) / 1e6:8.2f} ms")
