#!/bin/bash
# Placement probe: processes holding 0 / 16 / 48 GB of device memory while the engine allocates.
set -u
O=gpurun_out/${1:-r05_pl3}
mkdir -p $O
for rep in 1 2 3; do
  for h in 0 16 48; do
    PROBE_HOLD_GB=$h timeout -k 10 120 python tools/place_probe2.py >> $O/probe3.txt 2>&1 || { echo "STOP"; exit 1; }
    tail -1 $O/probe3.txt
  done
done
