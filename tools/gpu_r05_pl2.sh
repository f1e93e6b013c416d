#!/bin/bash
# Placement probe: alternating processes with / without a large allocation released before the
# engine is created (tools/place_probe2.py).  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_pl2}
mkdir -p $O
for rep in 1 2 3 4 5; do
  for pre in 0 96; do
    PROBE_PRE_GB=$pre timeout -k 10 120 python tools/place_probe2.py >> $O/probe2.txt 2>&1 || { echo "STOP"; exit 1; }
    tail -1 $O/probe2.txt
  done
done
