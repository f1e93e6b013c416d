#!/bin/bash
# Exchange-round class filter: GPU sharded tests, then the G = 8 per-rank probe with the
# filter (default filter_frac 0.3) and without it (filter_frac = 1).  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-xdfilt}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { echo "STOP tests"; tail -20 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 300 python -u tools/shard_probe.py 8 > $O/probe_G8.txt 2>&1 || { echo "STOP probe"; tail -5 $O/probe_G8.txt; exit 1; }
tail -17 $O/probe_G8.txt
timeout -k 10 300 python -u tools/shard_probe.py 8 24 xd_filter_frac=1 > $O/probe_G8_nofilter.txt 2>&1 || { echo "STOP probe nf"; exit 1; }
tail -1 $O/probe_G8_nofilter.txt
