#!/bin/bash
# Quick check of a kernel change under gpurun_out/$1: a pytest subset ($2, default the 2^27 one-engine
# parity test), the bench line without the CPU baseline, and the per-round split of the 2^27 bench.
set -u
O=gpurun_out/${1:-quick}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
T=${2:-tests/test_gpu_cfg4_full.py::test_cfg4_single_engine_equals_oracle}
if [ "$T" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $T -m gpu -v --timeout 300 --timeout-method thread -x > $O/pytest_gpu.txt 2>&1; ok $?
  tail -3 $O/pytest_gpu.txt
fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err; ok $?
python -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']; s=d.get('secondary',{})
print('2^27: %.3g nu/s, %.2f ms/step, dense %.0f us frac %.3f, dense_only %.0f us, sparse avg %.0f us' % (d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], r['dense_only']['avg_round_us'], r['sparse_rounds']['avg_round_us']))
print('2^24: %.3g nu/s, %.3f ms/step, dense %.0f us frac %.3f, sparse avg %.0f us' % (s['value'], s['ms_per_step'], s['avg_dense_round_us'], s['roofline_frac'], s['sparse_avg_round_us']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-dense-only --no-secondary > $O/prof.out 2>&1; ok $?
python tools/rounds.py $(find $O/prof -name '*kernel_trace.csv' | head -1) > $O/rounds.txt; ok $?
tail -17 $O/rounds.txt
echo done
