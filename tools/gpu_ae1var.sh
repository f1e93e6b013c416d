#!/bin/bash
# One-GPU ANTIENTROPY: GPU tests of the anti-entropy paths on the default library, then
# tools/ae_rounds.py (configs[4]) on it and on exp/ variants: VARS="a b" bash tools/gpu_ae1var.sh <out>
set -u
O=gpurun_out/${1:-ae1var}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -k "antientropy or ae_ or AE or cfg4" -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { echo "STOP tests"; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 200 python -u tools/ae_rounds.py > $O/default.txt 2>&1 || { echo "STOP default"; tail -5 $O/default.txt; exit 1; }
echo "== default"; tail -4 $O/default.txt
for X in ${VARS:-}; do
  GOSSIP_LIB=exp/lib$X.so timeout -k 10 200 python -u tools/ae_rounds.py > $O/$X.txt 2>&1 || { echo "STOP $X"; exit 1; }
  echo "== $X"; tail -4 $O/$X.txt
done
