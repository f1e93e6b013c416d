#!/bin/bash
# One GPU past the MALL: library variants (exp/lib<X>.so) on 2^26 and 2^27 nodes
# (parity: the GPU tests on the default build); prints the dense-round time per variant.
set -u
O=gpurun_out/${1:-big}; shift
mkdir -p $O
export TMPDIR=/tmp
for X in "$@"; do
  for LG in ${LGS:-26 27}; do
    GOSSIP_LIB=exp/lib$X.so EXP_N=$((1 << LG)) EXP_STEPS=3 timeout -k 10 300 python tools/exp_bench.py > $O/$X.$LG.txt 2>&1 || { echo "STOP $X $LG"; tail -3 $O/$X.$LG.txt; exit 1; }
    echo "$X 2^$LG: $(tail -1 $O/$X.$LG.txt)"
  done
done
