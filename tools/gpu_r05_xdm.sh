#!/bin/bash
# Filter-aware exchange-round cost in the link-aware plan: sharded / group / cfg4 GPU tests, then
# tools/shard_probe.py at G = 8 (and 4, 2) with the default plan.  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_xdm}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_group.py tests/test_gpu_multiprocess.py tests/test_gpu_cfg4_full.py -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest.txt 2>&1; ok $?
tail -1 $O/pytest.txt
for g in "8 24" "4 25" "2 26"; do
  set -- $g
  timeout -k 10 300 python tools/shard_probe.py $1 $2 > $O/probe_G$1.txt 2>&1; ok $?
  tail -1 $O/probe_G$1.txt
done
