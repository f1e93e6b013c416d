#!/bin/bash
# Round-5 end: tools/shard_probe.py per-rank device time at G = 2 x 2^26, 4 x 2^25, 8 x 2^24, with
# the link-aware plan (default) and the device-only plan (link_gbps=0).  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_probes}
mkdir -p $O
export TMPDIR=/tmp
for g in "2 26" "4 25" "8 24"; do
  set -- $g
  timeout -k 10 300 python tools/shard_probe.py $1 $2 > $O/probe_G$1.txt 2>&1 || { echo STOP; tail -5 $O/probe_G$1.txt; exit 1; }
  tail -2 $O/probe_G$1.txt
  timeout -k 10 300 python tools/shard_probe.py $1 $2 link_gbps=0 > $O/probe_G$1_devplan.txt 2>&1 || { echo STOP; exit 1; }
  tail -2 $O/probe_G$1_devplan.txt
done
