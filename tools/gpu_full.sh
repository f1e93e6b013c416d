#!/bin/bash
# GPU session: full GPU suite, smoke, bench, per-rank sharded probes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { echo "STOP: tests exited $rc"; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; ok $?
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; ok $?
cat gpurun_out/bench.json
for G in 2 4 8; do
  timeout -k 10 200 python -u tools/shard_probe.py $G > gpurun_out/probe_G$G.txt 2>&1; ok $?
  tail -1 gpurun_out/probe_G$G.txt
done
echo done
