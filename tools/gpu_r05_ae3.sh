#!/bin/bash
# Round 5: ANTIENTROPY rounds run one at a time clear their totals from the binned emit and read
# them back once (no memset, no second copy + sync per round).  The AE GPU tests, then
# tools/ae_step.py and a kernel trace with its idle gaps.  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_ae3}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_antientropy.py tests/test_gpu_ae_sharded.py -m gpu -v --timeout 300 --timeout-method thread -x > $O/pytest_ae.txt 2>&1; ok $?; tail -1 $O/pytest_ae.txt
for rep in 1 2; do
  AE_RUNS=3 timeout -k 10 300 python tools/ae_step.py > $O/ae_step.$rep.txt 2>&1; ok $?; tail -1 $O/ae_step.$rep.txt
done
AE_RUNS=3 AE_TIMING=0 timeout -k 10 300 python tools/ae_step.py > $O/ae_step_notiming.txt 2>&1; ok $?; tail -1 $O/ae_step_notiming.txt
AE_RUNS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/ae_step.py > $O/prof.out 2>&1; ok $?
F=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $F $O/kernel_stats.csv
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python tools/trace_gaps.py $T 3 > $O/gaps.txt; ok $?; head -8 $O/gaps.txt
echo done
