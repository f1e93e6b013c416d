#!/bin/bash
# Class-split dense rounds: parity at 2^27 / 2^26+4099, then step times for cls_frac 0 / 0.7 / 2 at
# configs[3] and a kernel trace split into rounds (default params).
set -u
O=gpurun_out/${1:-r04_b}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_faults.py -v --timeout 120 --timeout-method thread -x > $O/pytest_faults.txt 2>&1; ok $?
tail -1 $O/pytest_faults.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_cfg4_full.py -k "fixture or cls" -v --timeout 300 --timeout-method thread -x > $O/pytest_cls.txt 2>&1; ok $?
tail -3 $O/pytest_cls.txt
for c in 0 0.7 2; do
  EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=4 EXP_PARAMS=cls_frac=$c timeout -k 10 120 python -u tools/exp_bench.py > $O/exp_cls$c.txt 2>&1; ok $?
  cat $O/exp_cls$c.txt
done
EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=3 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/exp_bench.py > $O/prof.out 2>&1; ok $?
python tools/rounds.py $(find $O/prof -name '*kernel_trace.csv' | head -1) > $O/rounds.txt; ok $?
tail -16 $O/rounds.txt
