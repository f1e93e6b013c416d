#!/bin/bash
# serve ablations at 2^27, every round dense (timing / traffic only: B, D compute wrong results):
#   B no reply stores, C a reply in every slot (full senders' too), D no id loads (ids from the index)
set -u
O=gpurun_out/${1:-r04_n}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
for L in ${LIBS:-default exp/libsvB.so exp/libsvC.so exp/libsvD.so}; do
  T=$(basename $L .so)
  if [ $L = default ]; then V=""; else V="GOSSIP_LIB=$L"; fi
  E="EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_PARAMS=sparse_frac=-1"
  env $V $E EXP_STEPS=2 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k_$T -o run -- python tools/exp_bench.py > $O/k_$T.out 2>&1; ok $?
  grep "dense round" $O/k_$T.out
  python tools/kstats.py $(find $O/k_$T -name '*kernel_stats.csv' | head -1) bin_ > $O/kstats_$T.txt; cat $O/kstats_$T.txt
  env $V $E EXP_STEPS=1 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_$T -o fetch -- python tools/exp_bench.py > $O/pf_$T.out 2>&1; ok $?
  env $V $E EXP_STEPS=1 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_$T -o write -- python tools/exp_bench.py > $O/pw_$T.out 2>&1; ok $?
  python tools/pmc_dense.py $O/pmc_$T "2^27 $T" $O/pmc_$T.json > /dev/null; ok $?
  python -c "
import json; d=json.load(open('$O/pmc_$T.json')); N=1<<27
print('  rounds', d['dense_rounds_profiled'], {k: (round(v['fetch_corrected']/N,1), round(v['write']/N,1)) for k,v in d['per_kernel_bytes_per_dense_round'].items()})"
done
