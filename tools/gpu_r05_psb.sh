#!/bin/bash
# Placement calibration of the sharded state all-gather slab (place_sb): the sharded / group /
# multiprocess / configs[3] GPU tests, then tools/shard_probe.py at G = 2 x 2^26 and G = 4 x 2^25
# with place_tries 1 and the default.  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_psb}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_group.py tests/test_gpu_multiprocess.py tests/test_gpu_cfg4_full.py -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest.txt 2>&1; ok $?
tail -1 $O/pytest.txt
for g in "2 26" "4 25"; do
  set -- $g
  timeout -k 10 300 python tools/shard_probe.py $1 $2 place_tries=1 > $O/probe_G$1_p1.txt 2>&1; ok $?
  tail -2 $O/probe_G$1_p1.txt | head -1
  timeout -k 10 300 python tools/shard_probe.py $1 $2 > $O/probe_G$1.txt 2>&1; ok $?
  tail -2 $O/probe_G$1.txt | head -1
done
echo done
