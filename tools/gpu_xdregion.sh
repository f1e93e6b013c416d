#!/bin/bash
# Exchange-round sender regions: sharded GPU tests on the default library, then the G = 8 probe
# (tools/shard_probe.py) on exp/ variants: VARS="a b" bash tools/gpu_xdregion.sh <out>
set -u
O=gpurun_out/${1:-xdregion}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_multiprocess.py -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { echo "STOP tests"; tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for X in ${VARS:-}; do
  GOSSIP_LIB=exp/lib$X.so timeout -k 10 300 python -u tools/shard_probe.py 8 > $O/$X.txt 2>&1 || { echo "STOP $X"; tail -5 $O/$X.txt; exit 1; }
  echo "== $X"; grep -E "round  9 |rounds=" $O/$X.txt | cut -c1-260
done
