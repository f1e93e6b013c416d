#!/bin/bash
# stale-filtered binned dense ANTIENTROPY rounds without the peer probe, gated on the stale share
set -u
O=gpurun_out/${1:-r04_i}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_antientropy.py tests/test_gpu_ae_sharded.py -v --timeout 300 --timeout-method thread -x > $O/pytest_ae.txt 2>&1; ok $?
tail -3 $O/pytest_ae.txt
for P in "" ae_dense_filter=0 "" ae_dense_filter=0; do
  AE_PARAMS=$P AE_TIMING=0 timeout -k 10 200 python -u tools/ae_step.py > $O/ae.txt 2>&1; ok $?
  cat $O/ae.txt
done
python tools/ae_rounds.py > $O/ae_rounds.txt 2>&1; ok $?
head -16 $O/ae_rounds.txt; tail -4 $O/ae_rounds.txt
