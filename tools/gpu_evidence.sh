#!/bin/bash
# A full round record under gpurun_out/$1: GPU tests, smoke, the bench line (configs[3], 2^27 nodes on
# one GPU, with the configs[2] secondary), rocprof kernel trace + stats of the bench, per-round split,
# and PMC HBM traffic of the dense rounds (one counter group per pass) for both workloads.
# SKIP_TESTS=1 skips pytest + smoke; SKIP_PMC=1 the PMC passes.
set -u
O=gpurun_out/${1:-evidence}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -x > $O/pytest_gpu.txt 2>&1; ok $?
  tail -1 $O/pytest_gpu.txt
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; ok $?
  tail -1 $O/smoke.txt
fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err; ok $?
cat $O/bench.json
P="--no-cpu-baseline --no-dense-only --no-secondary --no-antientropy"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 $P > $O/prof.out 2>&1; ok $?
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv 2>/dev/null || find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
python tools/rounds.py $(find $O/prof -name '*kernel_trace.csv' | head -1) > $O/rounds.txt; ok $?
tail -18 $O/rounds.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof24 -o run -- python bench.py --nodes 16777216 --steps 20 --warmup 5 $P > $O/prof24.out 2>&1; ok $?
find $O/prof24 -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats_2p24.csv \;
python tools/rounds.py $(find $O/prof24 -name '*kernel_trace.csv' | head -1) > $O/rounds_2p24.txt; ok $?
tail -16 $O/rounds_2p24.txt
if [ "${SKIP_PMC:-0}" != "1" ]; then
  for n in 27 24; do
    B="python bench.py --nodes $((1 << n)) --steps 2 --warmup 1 --place-tries 1 $P"
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc$n -o fetch -- $B > $O/pmc_fetch$n.out 2>&1; ok $?
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc$n -o write -- $B > $O/pmc_write$n.out 2>&1; ok $?
    python tools/pmc_dense.py $O/pmc$n "pushpull k=2 R=64, 2^$n nodes over 1 GPU" $O/pmc_dense_2p$n.json; ok $?
  done
fi
echo done
