#!/bin/bash
# Binned sparse rounds: parity (every round binned, both commit modes, 2^24 / 2^25+ / 2^27),
# step times with and without them at configs[3], and a kernel trace split into rounds.
set -u
O=gpurun_out/${1:-r04_c}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_big_paths.py tests/test_gpu_cfg4_full.py -k "sparse_bs or fixture" -v --timeout 300 --timeout-method thread -x > $O/pytest_bs.txt 2>&1; ok $?
tail -3 $O/pytest_bs.txt
for c in 0 -1; do
  EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=4 EXP_PARAMS=sparse_bs=$c timeout -k 10 120 python -u tools/exp_bench.py > $O/exp_bs$c.txt 2>&1; ok $?
  cat $O/exp_bs$c.txt
done
EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=3 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/exp_bench.py > $O/prof.out 2>&1; ok $?
python tools/rounds.py $(find $O/prof -name '*kernel_trace.csv' | head -1) > $O/rounds.txt; ok $?
tail -16 $O/rounds.txt
