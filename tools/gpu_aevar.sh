#!/bin/bash
# Sharded ANTIENTROPY per-rank probe (tools/ae_shard_probe.py, G = 8) on the default library and
# on exp/ variants (tools/build_variants.sh): VARS="a b" bash tools/gpu_aevar.sh <out>
set -u
O=gpurun_out/${1:-aevar}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ae_shard_probe.py 8 > $O/default.txt 2>&1 || { echo "STOP default"; tail -5 $O/default.txt; exit 1; }
echo "== default"; grep -E "round  50|rounds=" $O/default.txt | cut -c1-240
for X in ${VARS:-}; do
  GOSSIP_LIB=exp/lib$X.so timeout -k 10 400 python -u tools/ae_shard_probe.py 8 > $O/$X.txt 2>&1 || { echo "STOP $X"; exit 1; }
  echo "== $X"; grep -E "round  50|rounds=" $O/$X.txt | cut -c1-240
done
