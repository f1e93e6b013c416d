#!/bin/bash
# Round 5: the queued scan in the sharded sparse rounds and the direct-round commit reading D only
# at S_t's nonzero nodes.  Sharded / group GPU tests and the one-engine sparse paths, then
# tools/shard_probe.py at G = 8 x 2^24 with and without the queue, and the per-round split of the
# 2^27 bench under rocprof.  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_sxq}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_group.py -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest_shard.txt 2>&1; ok $?
tail -1 $O/pytest_shard.txt
timeout -k 10 300 python tools/shard_probe.py 8 24 > $O/probe_G8.txt 2>&1; ok $?
tail -3 $O/probe_G8.txt
timeout -k 10 300 python tools/shard_probe.py 8 24 scan_queue=0 > $O/probe_G8_noq.txt 2>&1; ok $?
tail -3 $O/probe_G8_noq.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-dense-only --no-antientropy > $O/prof.out 2>&1; ok $?
T=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python tools/rounds.py $T > $O/rounds.txt; ok $?
python tools/sparse_rounds.py $T > $O/sparse_rounds.txt; ok $?
cat $O/sparse_rounds.txt
echo done
