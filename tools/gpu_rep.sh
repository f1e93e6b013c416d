#!/bin/bash
# Replicated dense rounds: the sharded GPU tests that run them, then the per-rank
# device-time probe and the gloo rehearsal lines at G = 2 and 4.  Every step under its own limit.
set -u
O=gpurun_out/${OUT:-rep}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: $2 exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_group.py tests/test_gpu_multiprocess.py -m gpu -v \
  --timeout 300 --timeout-method thread -x -k "${K:-replicat}" > $O/pytest_gpu.txt 2>&1
rc=$?; tail -4 $O/pytest_gpu.txt; ok $rc pytest
