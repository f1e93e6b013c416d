#!/bin/bash
# Sweeps one gossip_set_param knob on the bench workload (tools/exp_bench.py): $NAME over $VALUES at
# each size in $SIZES, twice, alternating.  Output under gpurun_out/$OUT.
set -u
O=gpurun_out/${OUT:-sweep}
mkdir -p $O
export TMPDIR=/tmp
for n in ${SIZES:-134217728}; do
  for rep in $(seq 1 ${REPS:-2}); do
    for v in ${VALUES}; do
      EXP_N=$n EXP_PARAMS="$NAME=$v" timeout -k 10 200 python tools/exp_bench.py > $O/$NAME.$v.$n.$rep.txt 2>&1 || { echo "STOP $v $n"; tail -5 $O/$NAME.$v.$n.$rep.txt; exit 1; }
      echo "n=$n $NAME=$v: $(tail -1 $O/$NAME.$v.$n.$rep.txt)"
    done
  done
done
