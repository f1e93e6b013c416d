#!/bin/bash
# Exchange dense rounds: GPU lockstep parity, then the per-rank probe at G = 8 and 4 (exchange) and
# G = 8 with the state all-gather, with a rocprofv3 kernel summary of the G = 8 exchange run.
set -u
O=gpurun_out/${1:-xd}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -m gpu -v --timeout 300 --timeout-method thread -x > $O/pytest_sharded.txt 2>&1
rc=$?; tail -5 $O/pytest_sharded.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/shard_probe.py 8 > $O/probe_G8_xd.txt 2>&1 || { tail $O/probe_G8_xd.txt; exit 1; }
tail -2 $O/probe_G8_xd.txt
timeout -k 10 300 python -u tools/shard_probe.py 4 > $O/probe_G4_xd.txt 2>&1 || { tail $O/probe_G4_xd.txt; exit 1; }
tail -1 $O/probe_G4_xd.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_G8 -o run -- python tools/shard_probe.py 8 > $O/prof_G8.out 2>&1 || exit 1
