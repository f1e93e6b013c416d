#!/bin/bash
# Sharded per-rank probe (tools/shard_probe.py) at G shards x 2^24 nodes, plus a rocprofv3 kernel
# trace + stats of the same run.  Usage: gpu_probe.sh <out> <G...>
set -u
O=gpurun_out/${1:-probe}; shift
mkdir -p $O
export TMPDIR=/tmp
for G in "$@"; do
  timeout -k 10 300 python -u tools/shard_probe.py $G > $O/probe_G$G.txt 2>&1 || { echo "STOP G=$G"; tail -5 $O/probe_G$G.txt; exit 1; }
  tail -3 $O/probe_G$G.txt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_G$G -o run -- python tools/shard_probe.py $G > $O/prof_G$G.out 2>&1 || { echo "STOP prof G=$G"; exit 1; }
done
