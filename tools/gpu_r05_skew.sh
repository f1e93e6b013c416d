#!/bin/bash
# Skew between the record slab's arrays (experiment builds exp/libsk*.so of a GOSSIP_EXP_SKEW macro in
# bin_carve, removed after this A/B: no skew helped), each process with the
# placement calibration on: dense round at 2^27 (tools/place_probe4.py), 3 processes per variant.
set -u
O=gpurun_out/${1:-r05_skew}
mkdir -p $O
for rep in 1 2 3; do
  for X in sk0 sk2k sk36k sk1m; do
    echo -n "$X " >> $O/probe.txt
    GOSSIP_LIB=exp/lib$X.so timeout -k 10 150 python tools/place_probe4.py >> $O/probe.txt 2>&1 || { echo "STOP"; tail -5 $O/probe.txt; exit 1; }
    tail -1 $O/probe.txt
  done
done
