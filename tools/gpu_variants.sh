#!/bin/bash
# Per-kernel dense-round times for library variants built into exp/lib<X>.so (tools/build_variants.sh).
set -u
mkdir -p gpurun_out/var
export TMPDIR=/tmp
for X in ${VARS}; do
  GOSSIP_LIB=exp/lib$X.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/var/$X -o run -- python tools/exp_rounds.py > gpurun_out/var/$X.out 2>&1 || { echo "STOP $X"; exit 1; }
  echo "== $X"; python tools/rounds.py gpurun_out/var/$X/run_kernel_trace.csv | grep -E "${GREP:-dense}" | tail -${TAILN:-4}
done
