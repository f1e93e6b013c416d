#!/bin/bash
# Which array of the record slab carries the dense round's placement mode: experiment builds (a
# GOSSIP_EXP_ARR macro in place_bins, removed after this measurement) whose
# trial rounds take only the masked arrays from each candidate (3 dst+src, 4 prec, 8 resp,
# 16 off+offT, 31 all), 8 candidates each, logged (tools/place_probe4.py).
set -u
O=gpurun_out/${1:-r05_arr}
mkdir -p $O
for rep in 1 2; do
  for X in arr3 arr4 arr8 arr16 arr31; do
    echo "== $X" >> $O/log.txt
    GOSSIP_LIB=exp/lib$X.so timeout -k 10 150 python tools/place_probe4.py >> $O/log.txt 2>&1 || { echo STOP; tail -5 $O/log.txt; exit 1; }
  done
done
grep -v "amdgpu.ids" $O/log.txt
