#!/bin/bash
# Round 5: serve's ids in long runs (param serve_lr): parity against the OpenMP oracle (2^25 and
# 2^26 + every round dense), the dense-round A/B at 2^27 and 2^26 (tools/exp_bench.py, alternating),
# and a rocprof kernel split of each at 2^27.  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_lr}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
for P in "serve_lr=1" "serve_lr=1 sparse_frac=-1"; do
  timeout -k 10 300 python tools/variant_parity.py 25 0x5EED0003 "$P" > $O/parity25.txt 2>&1; ok $?; tail -1 $O/parity25.txt
done
timeout -k 10 300 python tools/variant_parity.py 26 0x5EED0004 "serve_lr=1 sparse_frac=-1" > $O/parity26.txt 2>&1; ok $?; tail -1 $O/parity26.txt
for n in 134217728 67108864; do
  for rep in 1 2; do
    for v in 0 1; do
      EXP_N=$n EXP_SEED=0x5EED0004 EXP_PARAMS="serve_lr=$v" timeout -k 10 200 python tools/exp_bench.py > $O/ab.$v.$n.$rep.txt 2>&1; ok $?
      echo "n=$n serve_lr=$v: $(tail -1 $O/ab.$v.$n.$rep.txt)"
    done
  done
done
for v in 0 1; do
  EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=3 EXP_PARAMS="serve_lr=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- python tools/exp_bench.py > $O/prof$v.out 2>&1; ok $?
  python tools/kstats.py $O/prof$v > $O/kstats$v.txt 2>&1 || find $O/prof$v -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats$v.csv \;
done
find $O -name '*kernel_stats.csv' | head
echo done
