#!/bin/bash
# Round 4, first call: the GPU suite on the pruned tree, smoke, and a short bench (self-check).
set -u
O=gpurun_out/r04_a
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -x > $O/pytest_gpu.txt 2>&1; ok $?
tail -3 $O/pytest_gpu.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; ok $?
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dense-only > $O/bench.json 2> $O/bench.err; ok $?
cat $O/bench.json
