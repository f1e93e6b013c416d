#!/bin/bash
# Round 5: dynamic per-XCD tile queues in the persistent serve / apply (param tile_queues): parity
# against the OpenMP oracle (2^24 and 2^26, planned and every round dense), then the dense-round A/B
# (tools/exp_bench.py, alternating, 3 reps) at 2^27 and 2^24.  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_tq}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
for L in 24 26; do
  for P in "tile_queues=1" "tile_queues=1 sparse_frac=-1"; do
    timeout -k 10 300 python tools/variant_parity.py $L 0x5EED0004 "$P" > $O/parity$L.txt 2>&1; ok $?; tail -1 $O/parity$L.txt
  done
done
for n in 134217728 16777216; do
  for rep in 1 2 3; do
    for v in 0 1; do
      EXP_N=$n EXP_SEED=0x5EED0004 EXP_PARAMS="tile_queues=$v" timeout -k 10 200 python tools/exp_bench.py > $O/ab.$v.$n.$rep.txt 2>&1; ok $?
      echo "n=$n tile_queues=$v: $(tail -1 $O/ab.$v.$n.$rep.txt)"
    done
  done
done
echo done
