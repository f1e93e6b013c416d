#!/bin/bash
# Per-rank device time of the G = 2 plan at 2^27 nodes (tools/shard_probe.py, lockstep engines on one
# GPU), with the replicated dense rounds (default) and without them (replicate=0).
set -u
O=gpurun_out/${OUT:-rep_probe}
mkdir -p $O
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: $2 exited $rc"; exit "$rc"; fi; }
timeout -k 10 600 python -u tools/shard_probe.py 2 26 > $O/probe_G2.txt 2>&1; ok $? probe_G2
tail -4 $O/probe_G2.txt
timeout -k 10 600 python -u tools/shard_probe.py 2 26 replicate=0 > $O/probe_G2_norep.txt 2>&1; ok $? probe_G2_norep
tail -4 $O/probe_G2_norep.txt
