#!/bin/bash
# Pipelined ANTIENTROPY sparse rounds: parity (every path, the configs[4] fixture), then configs[4]
# to convergence with and without the pipeline (ae_ahead 1 / 8), wall and device time.
set -u
O=gpurun_out/${1:-r04_e}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_antientropy.py tests/test_gpu_ae_sharded.py tests/test_gpu_big_paths.py tests/test_gpu_cfg4_full.py -k "not G8" -v --timeout 300 --timeout-method thread -x > $O/pytest_ae.txt 2>&1; ok $?
tail -3 $O/pytest_ae.txt
for a in 1 8 1 8; do
  AE_AHEAD=$a timeout -k 10 200 python -u tools/ae_step.py > $O/ae_ahead$a.txt 2>&1; ok $?
  cat $O/ae_ahead$a.txt
done
AE_AHEAD=8 AE_TIMING=0 timeout -k 10 200 python -u tools/ae_step.py > $O/ae_ahead8_notiming.txt 2>&1; ok $?
cat $O/ae_ahead8_notiming.txt
# emit keeping the sender values in registers (exp/libkeep.so: no second read of S) vs the tree's
for L in default exp/libkeep.so exp/libu16.so exp/libkeep16.so default exp/libkeep.so exp/libu16.so exp/libkeep16.so; do
  if [ $L = default ]; then V=""; else V="GOSSIP_LIB=$L"; fi
  env $V EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=4 timeout -k 10 120 python -u tools/exp_bench.py > $O/exp_v.txt 2>&1; ok $?
  cat $O/exp_v.txt
done
# sparse rounds without the LDS summary (ns_frac 0.9 default) vs never (ns_frac 2)
for c in 2 0.9 2 0.9; do
  EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=4 EXP_PARAMS=ns_frac=$c timeout -k 10 120 python -u tools/exp_bench.py > $O/exp_ns.txt 2>&1; ok $?
  echo "ns_frac=$c $(cat $O/exp_ns.txt)"
done
EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=3 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/exp_bench.py > $O/prof.out 2>&1; ok $?
python tools/rounds.py $(find $O/prof -name '*kernel_trace.csv' | head -1) > $O/rounds.txt; ok $?
tail -16 $O/rounds.txt
