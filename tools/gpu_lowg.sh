#!/bin/bash
# Per-rank device time at G = 2 and 4 on the current tree (tools/shard_probe.py), plus sweeps of
# the sparse threshold for the all-gather rounds: output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-lowg}; mkdir -p $O
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
for G in 2 4; do
  timeout -k 10 200 python -u tools/shard_probe.py $G 24 > $O/probe_G$G.txt 2>&1; ok $?
  tail -1 $O/probe_G$G.txt
  for A in ${ARGS:-}; do
    timeout -k 10 200 python -u tools/shard_probe.py $G 24 $A > $O/probe_G${G}_$A.txt 2>&1; ok $?
    echo "$A: $(tail -1 $O/probe_G${G}_$A.txt)"
  done
done
