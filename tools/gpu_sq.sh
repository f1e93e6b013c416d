#!/bin/bash
# SQ/TA counter passes (one group per run) over a one-step bench; summary per kernel.
set -u
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-dense-only"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/sq -o sq1 -- $B > gpurun_out/sq/sq1.txt 2>&1; ok $?
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --kernel-trace --output-format csv -d gpurun_out/sq -o sq2 -- $B > gpurun_out/sq/sq2.txt 2>&1; ok $?
python tools/pmc_dispatch.py gpurun_out/sq frontier_scan > gpurun_out/sq/scan.txt; cat gpurun_out/sq/scan.txt
echo done
