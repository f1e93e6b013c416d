#!/bin/bash
# The replicated-round GPU tests, the placement parity test, then the G = 2 probe (tools/gpu_probe_rep.sh).
set -u
O=gpurun_out/${OUT:-rep2}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: $2 exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_group.py tests/test_gpu_multiprocess.py tests/test_gpu_parity.py -m gpu -v \
  --timeout 300 --timeout-method thread -x -k "replicat or placement" > $O/pytest_gpu.txt 2>&1
rc=$?; tail -3 $O/pytest_gpu.txt; ok $rc pytest
OUT=${OUT:-rep2} bash tools/gpu_probe_rep.sh; ok $? probe
