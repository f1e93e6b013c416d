#!/bin/bash
# Placement calibration with each candidate's trial time logged (exp/libplog.so, 8 tries).
set -u
O=gpurun_out/${1:-r05_pl6}
mkdir -p $O
for rep in 1 2 3; do
  GOSSIP_LIB=exp/libplog.so PROBE_TRIES=8 timeout -k 10 150 python tools/place_probe4.py >> $O/probe.txt 2>&1 || { echo "STOP"; tail -5 $O/probe.txt; exit 1; }
done
cat $O/probe.txt
