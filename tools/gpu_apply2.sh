#!/bin/bash
# Apply walk width x next-tile prefetch: per-kernel dense-round times for exp/lib<X>.so, each run twice.
set -u
mkdir -p gpurun_out/apply2
export TMPDIR=/tmp
O=gpurun_out/apply2
for X in u16p0 u8p4 u12p2 u8p0 u16p0 u8p4 u12p2 u8p0; do
  GOSSIP_LIB=exp/lib$X.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$X -o run -- python tools/exp_rounds.py > $O/$X.out 2>&1 || { echo "STOP $X"; exit 1; }
  echo "== $X"; python tools/rounds.py $O/$X/run_kernel_trace.csv | grep dense | tail -3
done
echo done
