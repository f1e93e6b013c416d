#!/bin/bash
# Placement calibration: 16 vs 8 candidates at 2^27 (3 processes each), and the trials' spread at
# 2^24 (logged build, 2 processes).
set -u
O=gpurun_out/${1:-r05_pl9}
mkdir -p $O
for rep in 1 2 3; do
  for t in 8 16; do
    PROBE_TRIES=$t timeout -k 10 200 python tools/place_probe4.py >> $O/probe.txt 2>&1 || { echo STOP; tail -5 $O/probe.txt; exit 1; }
    tail -1 $O/probe.txt
  done
done
for rep in 1 2; do
  PROBE_N=16777216 GOSSIP_LIB=exp/libplog.so timeout -k 10 200 python tools/place_probe4.py >> $O/log24.txt 2>&1 || { echo STOP; exit 1; }
done
grep -v amdgpu.ids $O/log24.txt
