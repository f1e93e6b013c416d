#!/bin/bash
# Round-2 evidence under gpurun_out/$1 (default r02): GPU tests, smoke, bench line, rocprof kernel
# trace + stats of the bench, PMC traffic of the dense rounds (one counter group per pass).
set -u
O=gpurun_out/${1:-r02}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; ok $?
  tail -1 $O/pytest_gpu.txt
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; ok $?
  tail -1 $O/smoke.txt
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; ok $?
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dense-only > $O/prof.out 2>&1; ok $?
python tools/rounds.py $O/prof/run_kernel_trace.csv > $O/rounds.txt; ok $?
tail -16 $O/rounds.txt
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dense-only"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc -o fetch -- $B > $O/pmc_fetch.out 2>&1; ok $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc -o write -- $B > $O/pmc_write.out 2>&1; ok $?
python tools/pmc_dense.py $O/pmc "pushpull k=2 R=64, 2^24 nodes/GPU x 1" $O/pmc_dense_round.json; ok $?
echo done
