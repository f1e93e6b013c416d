#!/bin/bash
# L2-window gather microbenchmark (tools/microbench6.hip), then the tree's 2^27 dense/sparse split
# with the emit keeping sender values in registers and the NS scan removed, and its parity.
set -u
O=gpurun_out/${1:-r04_f}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 300 ./exp/microbench6 > $O/microbench6.jsonl 2>&1; ok $?
cat $O/microbench6.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_big_paths.py tests/test_gpu_cfg4_full.py -k "not G8" -q --timeout 300 --timeout-method thread -x > $O/pytest.txt 2>&1; ok $?
tail -2 $O/pytest.txt
for i in 1 2; do
  EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=4 timeout -k 10 120 python -u tools/exp_bench.py > $O/exp_$i.txt 2>&1; ok $?
  cat $O/exp_$i.txt
done
