#!/bin/bash
# A GPU test subset (default: the one-shard round paths) plus the dense / sparse split at a few sizes.
#   bash tools/gpu_tests_subset.sh <out> ["pytest files"] ["sizes"]
set -u
O=gpurun_out/${1:-subset}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
T=${2:-tests/test_gpu_parity.py tests/test_gpu_big_paths.py tests/test_gpu_cfg4_full.py}
timeout -k 10 900 python -u -m pytest $T -k "not G8" -q --timeout 300 --timeout-method thread -x > $O/pytest.txt 2>&1; ok $?
tail -2 $O/pytest.txt
for n in ${3:-16777216 33554432 67108864 134217728}; do
  EXP_N=$n EXP_STEPS=4 timeout -k 10 120 python -u tools/exp_bench.py > $O/e.txt 2>&1; ok $?
  echo "N=$n $(grep -v amdgpu $O/e.txt)"
done
