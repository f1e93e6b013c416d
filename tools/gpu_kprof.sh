#!/bin/bash
# Per-kernel averages of library variants exp/lib<X>.so ($VARS, tools/build_variants.sh; X = default: the
# in-tree library) on the bench
# workload at each size in $SIZES: rocprofv3 --kernel-trace --stats over tools/exp_bench.py, then
# tools/kstats.py on the dense-round kernels.  Outputs under gpurun_out/$OUT.
set -u
O=gpurun_out/${OUT:-kprof}
mkdir -p $O
export TMPDIR=/tmp
for n in ${SIZES:-134217728}; do
  for X in ${VARS}; do
    D=$O/$X.$n
    L=exp/lib$X.so; [ "$X" = default ] && L=""
    GOSSIP_LIB=$L EXP_N=$n EXP_STEPS=${EXP_STEPS:-3} timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python tools/exp_bench.py > $D.txt 2>&1 || { echo "STOP $X $n"; tail -5 $D.txt; exit 1; }
    echo "== $X n=$n: $(grep 'per dense round' $D.txt)"
    python tools/kstats.py $(find $D -name '*kernel_stats.csv' | head -1) bin_ frontier_ transpose | tee $D.kstats
  done
done
echo done
