#!/bin/bash
# Round 5: configs[4] wall against device time (tools/ae_step.py, with and without the per-round
# events) and a rocprof kernel trace of one run.  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_ae}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
AE_RUNS=3 timeout -k 10 300 python tools/ae_step.py > $O/ae_step.txt 2>&1; ok $?; tail -1 $O/ae_step.txt
AE_RUNS=3 AE_TIMING=0 timeout -k 10 300 python tools/ae_step.py > $O/ae_step_notiming.txt 2>&1; ok $?; tail -1 $O/ae_step_notiming.txt
AE_RUNS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/ae_step.py > $O/prof.out 2>&1; ok $?
F=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $F $O/kernel_stats.csv; python tools/kstats.py $F > $O/kstats.txt; head -16 $O/kstats.txt
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); cp $T $O/kernel_trace.csv
echo done
