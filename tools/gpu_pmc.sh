#!/bin/bash
# PMC passes (one counter group per run) over a one-step bench: HBM bytes per round.
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-dense-only"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc -o fetch -- $B > gpurun_out/pmc/fetch.log 2>&1; ok $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc -o write -- $B > gpurun_out/pmc/write.log 2>&1; ok $?
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc -o hit -- $B > gpurun_out/pmc/hit.log 2>&1; ok $?
python tools/pmc_round.py gpurun_out/pmc "pushpull k=2 R=64, 2^24 nodes/GPU x 1" gpurun_out/pmc_round_kernel.json
echo done
