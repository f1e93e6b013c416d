#!/bin/bash
# Exchange-round send-slab placement (experiment build exp/libpxd.so of a GOSSIP_EXP_PLACE_XD block in
# xd_requests_enqueue, removed after this A/B: no modes) against the base library:
# tools/shard_probe.py 8 24 alternating, and one logged run.
set -u
O=gpurun_out/${1:-r05_pxd}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for X in base pxd; do
    GOSSIP_LIB=exp/lib$X.so timeout -k 10 300 python tools/shard_probe.py 8 24 > $O/probe_$X.$rep.txt 2>&1 || { echo STOP; tail -5 $O/probe_$X.$rep.txt; exit 1; }
    echo "$X $(tail -2 $O/probe_$X.$rep.txt | head -1)"
  done
done
GOSSIP_LIB=exp/libpxdlog.so timeout -k 10 300 python tools/shard_probe.py 8 24 > $O/probe_log.txt 2>&1 || exit 1
grep place_xd $O/probe_log.txt | head -24
