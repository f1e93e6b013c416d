#!/bin/bash
# GPU iteration: parity tests, bench, kernel trace with per-round breakdown.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
T=${TESTS:-tests/test_gpu_parity.py}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; ok $?
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; ok $?
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dense-only > gpurun_out/prof.out 2>&1; ok $?
python tools/rounds.py gpurun_out/prof/run_kernel_trace.csv; python tools/idle.py gpurun_out/prof/run_kernel_trace.csv | tail -3
echo done
