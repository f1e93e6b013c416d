#!/bin/bash
# Fused emit A/B (param fuse_emit): GPU parity tests, then dense-round timings and per-round
# kernel traces with and without it.  Output: gpurun_out/$1.
set -u
O=gpurun_out/${1:-fuse}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { echo "STOP tests"; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for P in fuse_emit=1 fuse_emit=0 fuse_emit=1 fuse_emit=0; do
  EXP_PARAMS=$P timeout -k 10 200 python tools/exp_bench.py > $O/t.txt 2>&1 || { echo "STOP $P"; cat $O/t.txt; exit 1; }
  echo "$P: $(cat $O/t.txt)"
done
for P in fuse_emit=1 fuse_emit=0; do
  EXP_PARAMS=$P EXP_STEPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$P -o run -- python tools/exp_bench.py > $O/$P.out 2>&1 || { echo "STOP prof $P"; exit 1; }
  echo "== $P"; python tools/rounds.py $O/$P/run_kernel_trace.csv | grep dense | tail -5
done
