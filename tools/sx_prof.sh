#!/bin/bash
# Kernel-level profile of sharded sparse rounds (8 shards x 2^22 on one GPU).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/sxprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sxprof -o run -- python tools/shard_probe.py 8 22 > gpurun_out/sxprof/out.txt 2>&1 || exit 1
cat gpurun_out/sxprof/out.txt | grep round
head -25 gpurun_out/sxprof/run_kernel_stats.csv
