#!/bin/bash
# Placement candidates 12 (default) vs 16 at 2^27, three processes each, alternating.
set -u
O=gpurun_out/${1:-r05_pl11}
mkdir -p $O
for rep in 1 2 3; do
  for t in 12 16; do
    PROBE_TRIES=$t timeout -k 10 200 python tools/place_probe4.py >> $O/probe.txt 2>&1 || { echo STOP; tail -5 $O/probe.txt; exit 1; }
    tail -1 $O/probe.txt
  done
done
