"""Average duration per (kernel, grid size) in a rocprofv3 kernel trace: tells apart
the passes of one kernel that run at different grids (e.g. the push and pull emit
passes of a sharded dense round)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
agg = defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    name = name.replace("gossip::", "")[:70]
    agg[(name, r.get("Grid_Size", r.get("Grid_Size_X", "?")))].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for (name, grid), d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(d)/1e3:9.3f} ms  n={len(d):5d}  avg={sum(d)/len(d):9.1f} us  grid={grid:>9}  {name}")
