#!/bin/bash
# ANTIENTROPY session: parity tests of every round path, then the configs[4] per-round profile
# under a kernel trace (tools/ae_rounds.py).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_antientropy.py tests/test_gpu_parity.py -k antientropy -x -v --timeout 300 --timeout-method thread > gpurun_out/ae_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ae_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ae_rounds.py 26 > gpurun_out/ae_rounds.txt 2>&1; rc=$?; tail -2 gpurun_out/ae_rounds.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/aeprof -o run -- python -u tools/ae_rounds.py 26 > gpurun_out/aeprof.log 2>&1
