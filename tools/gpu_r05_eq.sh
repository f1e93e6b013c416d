#!/bin/bash
# Round 5: the big emit's region queue (with tile_queues): parity (the configs[3] fixture at 2^27, the
# OpenMP oracle at 2^26 planned and every round dense), then the dense-round A/B at 2^27 (3 reps).
set -u
O=gpurun_out/${1:-r05_eq}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_cfg4_full.py -m gpu -v --timeout 300 --timeout-method thread -x -k "single_engine" > $O/pytest_cfg4.txt 2>&1; ok $?; tail -1 $O/pytest_cfg4.txt
for P in "tile_queues=1" "tile_queues=1 sparse_frac=-1"; do
  timeout -k 10 300 python tools/variant_parity.py 26 0x5EED0004 "$P" > $O/parity26.txt 2>&1; ok $?; tail -1 $O/parity26.txt
done
for rep in 1 2 3; do
  for v in 0 1; do
    EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_PARAMS="tile_queues=$v" timeout -k 10 200 python tools/exp_bench.py > $O/ab.$v.$rep.txt 2>&1; ok $?
    echo "tile_queues=$v: $(tail -1 $O/ab.$v.$rep.txt)"
  done
done
EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/exp_bench.py > $O/prof.out 2>&1; ok $?
F=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $F $O/kernel_stats.csv
echo done
