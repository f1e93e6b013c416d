#!/bin/bash
# GPU session: full GPU test suite, smoke, bench, rocprof stats, PMC traffic per round.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; ok $?
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; ok $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; ok $?
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1; ok $?
bash tools/gpu_pmc.sh
echo done
