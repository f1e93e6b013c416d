#!/bin/bash
# PMC passes (one counter group per run) over a short bench: HBM bytes + L2 hit rate per kernel.
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc -o fetch -- $B > gpurun_out/pmc/fetch.log 2>&1; ok $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc -o write -- $B > gpurun_out/pmc/write.log 2>&1; ok $?
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc -o hit -- $B > gpurun_out/pmc/hit.log 2>&1; ok $?
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace --output-format csv -d gpurun_out/pmc -o req -- $B > gpurun_out/pmc/req.log 2>&1; ok $?
echo done
