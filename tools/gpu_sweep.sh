#!/bin/bash
# Per-rank probe (tools/shard_probe.py, G shards x 2^24) for several knob sets.
# Usage: gpu_sweep.sh <out> <G> "<knobs>" ["<knobs>" ...]   (knobs: name=value ..., or "-")
set -u
O=gpurun_out/${1:-sweep}; G=$2; shift 2
mkdir -p $O
export TMPDIR=/tmp
i=0
for K in "$@"; do
  [ "$K" = "-" ] && K=""
  timeout -k 10 300 python -u tools/shard_probe.py $G 24 $K > $O/G${G}_$i.txt 2>&1 || { echo "STOP $K"; tail -3 $O/G${G}_$i.txt; exit 1; }
  echo "G=$G [$K] $(tail -1 $O/G${G}_$i.txt)"
  i=$((i+1))
done
