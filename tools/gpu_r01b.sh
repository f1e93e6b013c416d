#!/bin/bash
# GPU session: parity tests (both paths), smoke, bench, rocprof kernel stats.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 700 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; ok $?
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; ok $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err; ok $?
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1; ok $?
cat gpurun_out/prof/run_kernel_stats.csv | cut -c1-200
echo done
