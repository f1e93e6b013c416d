#!/bin/bash
# A/B of library variants exp/lib<X>.so (tools/build_variants.sh): a parity subset on the default
# library ($TESTS), then each variant's dense-round time at 2^24 and 2^27 (tools/exp_bench.py).
set -u
O=gpurun_out/${OUT:-ab}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest.txt 2>&1 || { echo "STOP tests"; tail -20 $O/pytest.txt; exit 1; }
  tail -1 $O/pytest.txt
fi
for n in ${SIZES:-16777216 134217728}; do
  for X in ${VARS}; do
    GOSSIP_LIB=exp/lib$X.so EXP_N=$n timeout -k 10 200 python tools/exp_bench.py > $O/$X.$n.txt 2>&1 || { echo "STOP $X $n"; cat $O/$X.$n.txt; exit 1; }
    echo "n=$n $(tail -1 $O/$X.$n.txt)"
  done
done
