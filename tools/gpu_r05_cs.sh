#!/bin/bash
# Round 5: bit-sliced per-rumor counts in the sparse commit (+ the queued scans).  Sparse-path,
# sharded and fault parity, the bench workload at 2^24 and 2^27 (tools/sweep_single.py), the
# per-round split of both sizes under rocprof, and shard_probe G = 8 with the device-only plan.
set -u
O=gpurun_out/${1:-r05_cs}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_big_paths.py tests/test_gpu_faults.py tests/test_gpu_cfg4_full.py tests/test_gpu_sharded.py -k "sparse or cfg4_single or auto or lockstep" -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest.txt 2>&1; ok $?
tail -1 $O/pytest.txt
SWEEP_N=16777216 SWEEP_STEPS=10 timeout -k 10 300 python tools/sweep_single.py - - - > $O/sweep.16777216.txt 2>&1; ok $?
cat $O/sweep.16777216.txt
SWEEP_N=134217728 SWEEP_STEPS=6 timeout -k 10 400 python tools/sweep_single.py - - > $O/sweep.134217728.txt 2>&1; ok $?
cat $O/sweep.134217728.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-dense-only --no-antientropy > $O/prof.out 2>&1; ok $?
T=$(find $O/prof -name '*kernel_trace.csv' | head -1)
python tools/rounds.py $T > $O/rounds.txt; ok $?
python tools/sparse_rounds.py $T > $O/sparse_rounds_2p24.txt; ok $?
cat $O/sparse_rounds_2p24.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof27 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dense-only --no-antientropy --no-secondary > $O/prof27.out 2>&1; ok $?
T=$(find $O/prof27 -name '*kernel_trace.csv' | head -1)
python tools/rounds.py $T > $O/rounds_2p27.txt; ok $?
python tools/sparse_rounds.py $T > $O/sparse_rounds_2p27.txt; ok $?
cat $O/sparse_rounds_2p27.txt
timeout -k 10 300 python tools/shard_probe.py 8 24 link_gbps=0 > $O/probe_G8_devplan.txt 2>&1; ok $?
tail -3 $O/probe_G8_devplan.txt
echo done
