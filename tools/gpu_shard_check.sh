#!/bin/bash
# Sharded GPU parity (lockstep, gloo multiprocess) then the G = 8 per-rank probe with kernel stats.
set -u
O=gpurun_out/${1:-shard}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_faults.py -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/shard_probe.py 8 > $O/probe_G8.txt 2>&1 || { tail $O/probe_G8.txt; exit 1; }
tail -1 $O/probe_G8.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_G8 -o run -- python tools/shard_probe.py 8 > $O/prof_G8.out 2>&1 || exit 1
