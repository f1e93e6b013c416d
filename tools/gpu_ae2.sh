#!/bin/bash
# GPU session: ANTIENTROPY parity (binned and direct sparse scans), configs[4] per-round profile, kernel trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_antientropy.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_ae.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_ae.log
[ $rc -ne 0 ] && { echo "STOP: tests exited $rc"; exit $rc; }
timeout -k 10 300 python -u tools/ae_rounds.py > gpurun_out/ae_rounds.txt 2>&1; ok $?
tail -5 gpurun_out/ae_rounds.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/aeprof -o ae -- python tools/ae_rounds.py > gpurun_out/aeprof.txt 2>&1; ok $?
python tools/ktrace_groups.py gpurun_out/aeprof/ae_kernel_trace.csv > gpurun_out/ae_kernels.txt
head -14 gpurun_out/ae_kernels.txt
echo done
