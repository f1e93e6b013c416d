#!/bin/bash
# Placement probe 3 (tools/place_probe3.py): which allocation carries the dense round's fast / slow
# mode — the bin slab (1), the state image (2), the frontier buffers (4), re-allocated in turn.
set -u
O=gpurun_out/${1:-r05_pl4}
mkdir -p $O
for m in 1 2 4; do
  GOSSIP_LIB=exp/librea.so PROBE_MASK=$m PROBE_TRIES=5 timeout -k 10 200 python tools/place_probe3.py >> $O/probe.txt 2>&1 || { echo "STOP"; tail -5 $O/probe.txt; exit 1; }
done
cat $O/probe.txt
