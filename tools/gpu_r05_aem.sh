#!/bin/bash
# Which ANTIENTROPY buffers carry the placement mode: experiment builds that re-allocate only the
# rows (aem1) or only the records (aem2) per candidate, each candidate's trial logged.
set -u
O=gpurun_out/${1:-r05_aem}
mkdir -p $O
for rep in 1 2; do
  for X in aem1 aem2; do
    echo "== $X" >> $O/log.txt
    GOSSIP_LIB=exp/lib$X.so timeout -k 10 300 python tools/ae_bench_line.py 1 >> $O/log.txt 2>&1 || { echo STOP; tail -5 $O/log.txt; exit 1; }
  done
done
grep -v "^{" $O/log.txt
python - $O/log.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print("ms_to_converge %.2f dense %.1f" % (d["ms_to_converge"], d["avg_dense_round_us"]))
PY
