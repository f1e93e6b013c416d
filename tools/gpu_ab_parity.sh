#!/bin/bash
# A/B of library variants exp/lib<X>.so ($VARS) with a parity check of each against the OpenMP
# oracle first (tools/variant_parity.py at 2^$PLOG nodes, every round dense and planned), then the
# dense-round times of tools/gpu_ab.sh.  Output under gpurun_out/$OUT.
set -u
O=gpurun_out/${OUT:-abp}
mkdir -p $O
export TMPDIR=/tmp
for X in ${VARS}; do
  for P in "sparse_frac=-1" ""; do
    GOSSIP_LIB=exp/lib$X.so timeout -k 10 300 python tools/variant_parity.py ${PLOG:-22} 0x5EED0003 "$P" > $O/parity_$X.txt 2>&1 || { echo "STOP parity $X"; tail -5 $O/parity_$X.txt; exit 1; }
    tail -1 $O/parity_$X.txt
    grep -q "parity OK" $O/parity_$X.txt || { echo "STOP mismatch $X"; exit 1; }
  done
done
OUT=${OUT:-abp} bash tools/gpu_ab.sh
