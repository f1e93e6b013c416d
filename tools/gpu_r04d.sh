#!/bin/bash
# Tile order of the persistent serve / apply (tile_map 0: XCD-contiguous ranges, 1: the chip on
# consecutive tiles) at configs[3] and configs[2], per-kernel times from a kernel trace.
set -u
O=gpurun_out/${1:-r04_d}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
for n in 134217728 16777216; do
  for m in 0 1 0 1; do
    EXP_N=$n EXP_SEED=0x5EED0004 EXP_STEPS=4 EXP_PARAMS=tile_map=$m timeout -k 10 120 python -u tools/exp_bench.py > $O/exp_$n.$m.txt 2>&1; ok $?
    echo "$n tile_map=$m: $(cat $O/exp_$n.$m.txt)"
  done
done
for m in 0 1; do
  EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=3 EXP_PARAMS=tile_map=$m timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$m -o run -- python tools/exp_bench.py > $O/prof$m.out 2>&1; ok $?
  python tools/rounds.py $(find $O/prof$m -name '*kernel_trace.csv' | head -1) > $O/rounds$m.txt; ok $?
  grep dense $O/rounds$m.txt | tail -3
done
