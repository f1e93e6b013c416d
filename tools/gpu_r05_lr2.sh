#!/bin/bash
# Round 5: the A/B of serve's long-run ids (param serve_lr) at 2^27 after the regroup kernel's
# batched loads: parity at 2^25 (every round dense) against the OpenMP oracle, the dense-round time
# (tools/exp_bench.py, alternating), rocprof kernel stats, and per variant the PMC passes (FETCH_SIZE,
# WRITE_SIZE; SQ / TCP / TCC groups of tools/gpu_pmc_sq.sh).  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_lr2}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 300 python tools/variant_parity.py 25 0x5EED0003 "serve_lr=1 sparse_frac=-1" > $O/parity25.txt 2>&1; ok $?; tail -1 $O/parity25.txt
for rep in 1 2; do
  for v in 0 1; do
    EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_PARAMS="serve_lr=$v" timeout -k 10 200 python tools/exp_bench.py > $O/ab.$v.$rep.txt 2>&1; ok $?
    echo "serve_lr=$v: $(tail -1 $O/ab.$v.$rep.txt)"
  done
done
for v in 0 1; do
  export EXP_N=134217728 EXP_SEED=0x5EED0004 EXP_STEPS=2 EXP_PARAMS="serve_lr=$v"
  B="python tools/exp_bench.py"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o run -- $B > $O/prof$v.out 2>&1; ok $?
  F=$(find $O/prof$v -name "*kernel_stats.csv" | head -1); cp $F $O/kernel_stats$v.csv; python tools/kstats.py $F | head -7
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc$v -o fetch -- $B > $O/pmc_fetch$v.out 2>&1; ok $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc$v -o write -- $B > $O/pmc_write$v.out 2>&1; ok $?
  python tools/pmc_dense.py $O/pmc$v "serve_lr=$v, pushpull k=2 R=64, 2^27 nodes" $O/pmc_dense_lr$v.json; ok $?
  BENCH="$B" PMC_NODES=134217728 bash tools/gpu_pmc_sq.sh r05_lr2/sq$v; ok $?
  cp gpurun_out/r05_lr2/sq$v/pmc_sq.json $O/pmc_sq_lr$v.json
done
echo done
