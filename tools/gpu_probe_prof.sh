#!/bin/bash
set -u
O=gpurun_out/r04_aj
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/shard_probe.py 8 > $O/probe.txt 2>&1 || { echo STOP; tail -5 $O/probe.txt; exit 1; }
tail -3 $O/probe.txt
python tools/kstats.py $(find $O/prof -name '*kernel_stats.csv' | head -1) > $O/kstats.txt; head -40 $O/kstats.txt
