#!/bin/bash
# Placement at 2^24: up to 2.5x the candidates for small slabs (an experiment build of place_slab, not
# kept; 23 at 0.7 GB)
# against 12 (place_tries 12 caps the scaling? no: PROBE_TRIES=1 baseline and default), processes
# alternating; then the bench's configs[2] line twice.
set -u
O=gpurun_out/${1:-r05_pl12}
mkdir -p $O
for rep in 1 2 3; do
  PROBE_N=16777216 timeout -k 10 200 python tools/place_probe4.py >> $O/probe.txt 2>&1 || { echo STOP; tail -5 $O/probe.txt; exit 1; }
  tail -1 $O/probe.txt
  PROBE_N=16777216 PROBE_TRIES=1 timeout -k 10 200 python tools/place_probe4.py >> $O/probe.txt 2>&1 || { echo STOP; exit 1; }
  tail -1 $O/probe.txt
done
