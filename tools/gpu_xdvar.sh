#!/bin/bash
# Exchange-round kernel variants (exp/lib<X>.so): the G = 8 probe with every dense round an exchange
# round (sparse_frac=-1), under a rocprofv3 kernel summary.  Usage: gpu_xdvar.sh <out> <X...>
set -u
O=gpurun_out/${1:-xdvar}; shift
mkdir -p $O
export TMPDIR=/tmp
for X in "$@"; do
  GOSSIP_LIB=exp/lib$X.so timeout -k 10 120 python tools/xd_variant_check.py > $O/$X.check 2>&1 || { echo "CHECK $X"; tail -3 $O/$X.check; exit 1; }
  GOSSIP_LIB=exp/lib$X.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$X -o run -- python tools/shard_probe.py 8 24 sparse_frac=-1 > $O/$X.out 2>&1 || { echo "STOP $X"; tail -3 $O/$X.out; exit 1; }
  echo "== $X"; tail -1 $O/$X.out
done
