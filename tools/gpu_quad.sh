#!/bin/bash
# Quad run walkers: GPU parity tests on the default build, then dense-round timings of the
# exp/ variants (tools/build_variants.sh) and G = 8 probes over filter_frac.  Output: gpurun_out/$1.
set -u
O=gpurun_out/${1:-quad}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { echo "STOP tests"; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for X in ${VARS:-base quad}; do
  GOSSIP_LIB=exp/lib$X.so timeout -k 10 200 python tools/exp_bench.py > $O/$X.timer 2>&1 || { echo "STOP $X"; cat $O/$X.timer; exit 1; }
  cat $O/$X.timer
done
for X in ${VARS:-base quad}; do
  GOSSIP_LIB=exp/lib$X.so EXP_STEPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$X -o run -- python tools/exp_bench.py > $O/$X.out 2>&1 || { echo "STOP prof $X"; exit 1; }
  echo "== $X"; python tools/rounds.py $O/$X/run_kernel_trace.csv | grep dense | tail -5
done
for F in ${FILTS:-}; do
  timeout -k 10 300 python -u tools/shard_probe.py 8 24 xd_filter_frac=$F > $O/probe_G8_f$F.txt 2>&1 || { echo "STOP probe $F"; exit 1; }
  echo "xd_filter_frac=$F"; grep -E "xdense" $O/probe_G8_f$F.txt | cut -c1-200; tail -1 $O/probe_G8_f$F.txt
done
