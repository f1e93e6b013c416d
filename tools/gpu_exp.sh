#!/bin/bash
# timing experiments (GOSSIP_EXPERIMENT bits): kernel trace of one bench step per setting
set -u
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
for X in ${EXPS:-0 1 2 3}; do
  GOSSIP_EXPERIMENT=$X timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/exp/x$X -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-dense-only > gpurun_out/exp/x$X.out 2>&1 || { echo "STOP x$X"; exit 1; }
  echo "== exp $X"; python tools/rounds.py gpurun_out/exp/x$X/run_kernel_trace.csv | grep dense | head -3
done
