#!/bin/bash
# Round 5: the queued sparse scan (param scan_queue).  Parity of every sparse path (incl. the
# unqueued one) at configs[1..2] sizes, 2^25 + 4099 and configs[3]; then the bench workload at 2^24
# and 2^27 with and without the queue (tools/sweep_single.py), and the per-round split of the
# 2^27 bench under rocprof.  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_sq}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_big_paths.py tests/test_gpu_faults.py tests/test_gpu_cfg4_full.py -k "sparse or cfg4_single or auto" -m gpu -v --timeout 300 --timeout-method thread -x > $O/pytest.txt 2>&1; ok $?
tail -1 $O/pytest.txt
for n in 16777216 134217728; do
  SWEEP_N=$n SWEEP_STEPS=6 timeout -k 10 300 python tools/sweep_single.py - "scan_queue=0" - "scan_queue=0" ${EXTRA:-} > $O/sweep.$n.txt 2>&1; ok $?
  cat $O/sweep.$n.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-dense-only --no-secondary --no-antientropy > $O/prof.out 2>&1; ok $?
T=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python tools/rounds.py $T > $O/rounds.txt; ok $?
python tools/sparse_rounds.py $T > $O/sparse_rounds.txt; ok $?
cat $O/sparse_rounds.txt
cp $(find $O/prof -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv
echo done
