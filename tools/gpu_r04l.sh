#!/bin/bash
# Non-temporal loads of the tile images (serve / apply) at 2^27 against the tree: kernel times and
# the dense round's FETCH / WRITE per kernel.
set -u
O=gpurun_out/${1:-r04_l}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
for L in default exp/libtilent.so; do
  T=$(basename $L .so)
  if [ $L = default ]; then V=""; else V="GOSSIP_LIB=$L"; fi
  env $V EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=3 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$T -o run -- python tools/exp_bench.py > $O/k_$T.out 2>&1; ok $?
  grep "dense round" $O/k_$T.out
  python tools/kstats.py $(find $O/k_$T -name '*kernel_stats.csv' | head -1) bin_ > $O/kstats_$T.txt; cat $O/kstats_$T.txt
  env $V EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_$T -o fetch -- python tools/exp_bench.py > $O/pf_$T.out 2>&1; ok $?
  env $V EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_$T -o write -- python tools/exp_bench.py > $O/pw_$T.out 2>&1; ok $?
  python tools/pmc_dense.py $O/pmc_$T "2^27 $T" $O/pmc_$T.json; ok $?
done
