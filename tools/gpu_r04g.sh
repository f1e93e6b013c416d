#!/bin/bash
# ANTIENTROPY: one Philox call per node for churn + peer (timing variant exp/libaechurn.so) against the
# tree; the tree's configs[4] kernel split (rocprof); configs[2] (2^24) per-round split.
set -u
O=gpurun_out/${1:-r04_g}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
for L in default exp/libaechurn.so default exp/libaechurn.so; do
  if [ $L = default ]; then V=""; else V="GOSSIP_LIB=$L"; fi
  env $V AE_TIMING=0 timeout -k 10 200 python -u tools/ae_step.py > $O/ae.txt 2>&1; ok $?
  cat $O/ae.txt
done
AE_RUNS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/aeprof -o run -- python tools/ae_step.py > $O/aeprof.out 2>&1; ok $?
python tools/kstats.py $(find $O/aeprof -name '*kernel_stats.csv' | head -1) > $O/ae_kstats.txt 2>&1; cat $O/ae_kstats.txt | head -30
EXP_N=16777216 EXP_STEPS=4 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof24 -o run -- python tools/exp_bench.py > $O/prof24.out 2>&1; ok $?
cat $O/prof24.out | grep -v amdgpu
python tools/rounds.py $(find $O/prof24 -name '*kernel_trace.csv' | head -1) > $O/rounds24.txt; ok $?
tail -18 $O/rounds24.txt
