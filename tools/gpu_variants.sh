#!/bin/bash
# Dense-round times of library variants exp/lib<X>.so (tools/build_variants.sh) on the bench workload:
# engine timer (hipEvents) per variant, then a rocprofv3 kernel trace split into rounds.
set -u
O=gpurun_out/${OUT:-var}
mkdir -p $O
export TMPDIR=/tmp
for X in ${VARS}; do
  GOSSIP_LIB=exp/lib$X.so timeout -k 10 200 python tools/exp_bench.py > $O/$X.timer 2>&1 || { echo "STOP $X"; cat $O/$X.timer; exit 1; }
  cat $O/$X.timer
done
for X in ${VARS}; do
  GOSSIP_LIB=exp/lib$X.so EXP_STEPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$X -o run -- python tools/exp_bench.py > $O/$X.out 2>&1 || { echo "STOP $X"; exit 1; }
  echo "== $X"; python tools/rounds.py $O/$X/run_kernel_trace.csv | grep -E "${GREP:-dense}" | tail -${TAILN:-5}
done
