#!/bin/bash
# GPU session: parity tests, bench, kernel trace, SQ/TA counters.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; ok $?
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; ok $?
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1; ok $?
python tools/rounds.py gpurun_out/prof/run_kernel_trace.csv | tail -16
if [ "${SQ:-0}" = "1" ]; then bash tools/gpu_sq.sh; fi
echo done
