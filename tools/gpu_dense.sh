#!/bin/bash
# GPU session: dense-pipeline change — parity (one GPU + sharded), bench with the all-dense run, kernel trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_faults.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dense.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_dense.log
[ $rc -ne 0 ] && { echo "STOP: tests exited $rc"; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_dense.json 2> gpurun_out/bench.err; ok $?
python -c "import json; d=json.load(open('gpurun_out/bench_dense.json')); r=d['roofline']; print(round(d['value']/1e9,2), 'G', round(d['ms_per_step'],3), 'ms; dense-only round', round(r['dense_only']['avg_round_us'],1), 'us')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dense-only > gpurun_out/prof.log 2>&1; ok $?
python tools/rounds.py gpurun_out/prof/run_kernel_trace.csv | tail -16
echo done
