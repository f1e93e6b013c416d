#!/bin/bash
# ANTIENTROPY churn word from the first peer draw + stale-filtered binned dense rounds: parity (every
# path, the regenerated configs[4] fixture), configs[4] with the filter on / off, kernel split.
set -u
O=gpurun_out/${1:-r04_h}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_antientropy.py tests/test_gpu_ae_sharded.py -v --timeout 300 --timeout-method thread -x > $O/pytest_ae.txt 2>&1; ok $?
tail -3 $O/pytest_ae.txt
for P in "" ae_dense_filter=0 "" ae_dense_filter=0; do
  AE_PARAMS=$P AE_TIMING=0 timeout -k 10 200 python -u tools/ae_step.py > $O/ae.txt 2>&1; ok $?
  cat $O/ae.txt
done
AE_TIMING=1 timeout -k 10 200 python -u tools/ae_step.py > $O/ae_timing.txt 2>&1; ok $?
cat $O/ae_timing.txt
AE_RUNS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/aeprof -o run -- python tools/ae_step.py > $O/aeprof.out 2>&1; ok $?
python tools/kstats.py $(find $O/aeprof -name '*kernel_stats.csv' | head -1) > $O/ae_kstats.txt 2>&1; head -8 $O/ae_kstats.txt
python tools/ae_rounds.py > $O/ae_rounds.txt 2>&1; ok $?
head -16 $O/ae_rounds.txt
# run-bound prefetch in the binned walkers (tree) against the walkers without it (exp/libnopf.so)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_big_paths.py -q --timeout 300 --timeout-method thread -x > $O/pytest_pp.txt 2>&1; ok $?
tail -2 $O/pytest_pp.txt
for L in default exp/libnopf.so default exp/libnopf.so; do
  if [ $L = default ]; then V=""; else V="GOSSIP_LIB=$L"; fi
  env $V EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=3 timeout -k 10 120 python -u tools/exp_bench.py > $O/exp27.txt 2>&1; ok $?
  cat $O/exp27.txt
  env $V EXP_N=16777216 EXP_STEPS=6 timeout -k 10 120 python -u tools/exp_bench.py > $O/exp24.txt 2>&1; ok $?
  cat $O/exp24.txt
done
