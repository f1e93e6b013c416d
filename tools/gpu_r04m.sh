#!/bin/bash
# ANTIENTROPY binned sparse scan: 4 (tree) / 8 / 16 records in flight per lane
set -u
O=gpurun_out/${1:-r04_m}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
for L in default exp/libaescan8.so exp/libaescan16.so default exp/libaescan8.so exp/libaescan16.so; do
  if [ $L = default ]; then V=""; else V="GOSSIP_LIB=$L"; fi
  env $V AE_TIMING=0 timeout -k 10 200 python -u tools/ae_step.py > $O/ae.txt 2>&1; ok $?
  cat $O/ae.txt
done
for L in default exp/libaescan8.so exp/libaescan16.so; do
  T=$(basename $L .so)
  if [ $L = default ]; then V=""; else V="GOSSIP_LIB=$L"; fi
  env $V AE_RUNS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$T -o run -- python tools/ae_step.py > $O/p_$T.out 2>&1; ok $?
  echo $T; python tools/kstats.py $(find $O/p_$T -name '*kernel_stats.csv' | head -1) ae_bin
done
