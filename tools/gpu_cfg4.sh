#!/bin/bash
# configs[3] at full size (tests/test_gpu_cfg4_full.py) plus a timing of one 2^27-node engine.
set -u
O=gpurun_out/${1:-cfg4}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_cfg4_full.py -v --timeout 600 --timeout-method thread --durations=0 > $O/pytest_cfg4.txt 2>&1; ok $?
tail -12 $O/pytest_cfg4.txt
echo done
