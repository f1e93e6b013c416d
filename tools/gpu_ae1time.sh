#!/bin/bash
# tools/ae_rounds.py (configs[4], one GPU) on exp/ library variants, timing only:
# VARS="a b" bash tools/gpu_ae1time.sh <out>
set -u
O=gpurun_out/${1:-ae1time}
mkdir -p $O
for X in ${VARS:-}; do
  GOSSIP_LIB=exp/lib$X.so timeout -k 10 200 python -u tools/ae_rounds.py > $O/$X.txt 2>&1 || { echo "STOP $X"; tail -5 $O/$X.txt; exit 1; }
  echo "== $X"; tail -4 $O/$X.txt | head -3
done
