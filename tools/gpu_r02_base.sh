#!/bin/bash
# Round-2 baseline on a fresh box: bench line (driver defaults) + kernel trace of a short run.
set -u
mkdir -p gpurun_out/r02_base
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r02_base/bench.json 2> gpurun_out/r02_base/bench.err; ok $?
cat gpurun_out/r02_base/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_base/prof -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dense-only > gpurun_out/r02_base/prof.log 2>&1; ok $?
python tools/rounds.py gpurun_out/r02_base/prof/run_kernel_trace.csv > gpurun_out/r02_base/rounds.txt; ok $?
tail -20 gpurun_out/r02_base/rounds.txt
echo done
