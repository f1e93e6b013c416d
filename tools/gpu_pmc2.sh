#!/bin/bash
# DRAM traffic per kernel on dense rounds (tools/exp_rounds.py): one counter group per pass.
set -u
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
B="python tools/exp_rounds.py"
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc2 -o fetch -- $B > gpurun_out/pmc2/fetch.txt 2>&1; ok $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc2 -o write -- $B > gpurun_out/pmc2/write.txt 2>&1; ok $?
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --kernel-trace --output-format csv -d gpurun_out/pmc2 -o hit -- $B > gpurun_out/pmc2/hit.txt 2>&1; ok $?
for k in bin_emit bin_serve bin_apply; do echo "== $k"; python tools/pmc_dispatch.py gpurun_out/pmc2 $k | tail -3; done
echo done
