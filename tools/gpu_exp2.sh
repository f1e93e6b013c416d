#!/bin/bash
set -u
mkdir -p gpurun_out/exp2
export TMPDIR=/tmp
for X in ${EXPS}; do
  GOSSIP_EXPERIMENT=$X timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/exp2/x$X -o run -- python tools/exp_rounds.py > gpurun_out/exp2/x$X.out 2>&1 || { echo "STOP x$X"; exit 1; }
  echo "== exp $X"; python tools/rounds.py gpurun_out/exp2/x$X/run_kernel_trace.csv | grep dense | tail -3
done
