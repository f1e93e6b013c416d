#!/bin/bash
# GPU tests only (optionally a subset: $2 = pytest args), output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-tests}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${2:-tests} -m gpu -v --timeout 300 --timeout-method thread -x > $O/pytest_gpu.txt 2>&1
rc=$?
tail -25 $O/pytest_gpu.txt
exit $rc
