#!/bin/bash
# GPU session: sharded dense rounds on the binned passes — parity tests, per-rank probes, G=8 kernel trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_faults.py tests/test_gpu_multiprocess.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sb.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_sb.log
[ $rc -ne 0 ] && { echo "STOP: tests exited $rc"; exit $rc; }
for G in 2 4 8; do
  timeout -k 10 200 python -u tools/shard_probe.py $G > gpurun_out/probe_G$G.txt 2>&1; ok $?
  tail -1 gpurun_out/probe_G$G.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sbprof -o g8 -- python tools/shard_probe.py 8 > gpurun_out/sbprof_g8.txt 2>&1; ok $?
python tools/ktrace_groups.py gpurun_out/sbprof/g8_kernel_trace.csv > gpurun_out/sbprof_g8_groups.txt
head -16 gpurun_out/sbprof_g8_groups.txt
echo done
