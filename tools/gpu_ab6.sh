#!/bin/bash
# Round-6 A/B launcher (replaces the one-script-per-profile gpu_r05_*.sh launchers; they are in git
# history at 233a6c4).  Every step runs under its own time limit and the first failure ends the run.
#   OUT    output directory under gpurun_out/ (default ab6)
#   TESTS  pytest targets run first ("none": skip)
#   VARS   library variants: default (the in-tree library) or X = exp/libX.so (tools/build_variants.sh),
#          or p:name=value[,name=value] = the in-tree library with those gossip_set_param knobs
#   SIZES  node counts of the dense-round A/B (tools/exp_bench.py, every round as planned)
#   STEPS  bench steps per variant and size (default 4; the first is untimed)
#   KPROF  1: per-kernel rocprofv3 --stats of each variant and size (default 1)
#   PMC    1: HBM bytes and L2 request counters of each variant's dense rounds (one pass per counter
#          group, tools/pmc_dense.py + tools/pmc_sq.py), with placement trials off (place_tries 1)
#   LIST   1: rocprofv3 --list-avail into $OUT/counters.txt
#   PROBES "G log2N,...": tools/shard_probe.py per-rank device time (PROBE_LIB: a variant)
#   REH    1: gloo rehearsals of bench.py --gpus 2 and 4 on the one GPU (the N > 1 line's fields)
#   SEQ    "N:engines,...": placement over engines made one after another (tools/place_seq.py)
#   SKIP_AB 1: stop before the per-variant A/B
#   PLACE  1: TLB / L2 / DRAM-credit counters of every placement candidate's trial rounds at 2^27
#          (tools/place_probe4.py under rocprofv3 --pmc, one pass per group; tools/place_pmc.py), with
#          the library PLACE_LIB (default: the in-tree one)
set -u
O=gpurun_out/${OUT:-ab6}
mkdir -p $O $O/place
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: $2 exited $rc"; exit "$rc"; fi; }
if [ "${LIST:-0}" = 1 ]; then
  timeout -k 10 120 rocprofv3 --list-avail > $O/counters.txt 2>&1; ok $? list-avail
fi
if [ "${PLACE:-0}" = 1 ]; then  # counters of each placement candidate's trial rounds (tools/place_pmc.py)
  L=exp/lib${PLACE_LIB:-default}.so; [ "${PLACE_LIB:-default}" = default ] && L=""
  i=0
  for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_THRASHING_STALL_sum" \
             "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_STALL_sum" \
             "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum" \
             "TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    GOSSIP_LIB=$L PROBE_TRIES=12 timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv \
      -d $O/place/p$i -o p -- python tools/place_probe4.py > $O/place/p$i.txt 2>&1; ok $? "place pass $i"
    tail -1 $O/place/p$i.txt
  done
  python tools/place_pmc.py $O/place 12 > $O/place/summary.txt; ok $? place_pmc
  grep -E "^==|r\(" $O/place/summary.txt
fi
if [ "${TESTS:-none}" != none ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread -x \
    -p no:cacheprovider > $O/pytest_gpu.txt 2>&1
  rc=$?; tail -4 $O/pytest_gpu.txt; ok $rc pytest
fi
if [ -n "${SEQ:-}" ]; then  # placement over engines made one after another: "N:engines,..." (tools/place_seq.py)
  IFS=, read -ra SS <<< "$SEQ"
  for q in "${SS[@]}"; do
    PROBE_N=${q%%:*} PROBE_ENGINES=${q##*:} timeout -k 10 600 python -u tools/place_seq.py > $O/place_seq_${q%%:*}.txt 2>&1
    ok $? "place_seq $q"
    cat $O/place_seq_${q%%:*}.txt
  done
fi
if [ -n "${PROBES:-}" ]; then  # per-rank device time of sharded rounds: "G log2N" pairs, comma-separated
  IFS=, read -ra PS <<< "$PROBES"
  for g in "${PS[@]}"; do
    set -- $g
    GOSSIP_LIB=${PROBE_LIB:-} timeout -k 10 300 python tools/shard_probe.py $1 $2 > $O/probe_G$1.txt 2>&1; ok $? "probe $g"
    tail -2 $O/probe_G$1.txt
  done
fi
if [ "${REH:-0}" = 1 ]; then  # gloo rehearsals of the N > 1 bench line on one GPU (not a measurement)
  for G in 2 4; do
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $G --master-addr 127.0.0.1 \
      --master-port $((29515 + G)) bench.py --gpus $G --steps 2 --warmup 1 --backend gloo \
      > $O/bench_rehearsal_gloo_G$G.json 2> $O/rehearsal_G$G.err; ok $? "rehearsal G=$G"
    cat $O/bench_rehearsal_gloo_G$G.json
  done
fi
if [ "${SKIP_AB:-0}" = 1 ]; then echo done; exit 0; fi
for n in ${SIZES:-134217728}; do
  for X in ${VARS:-default}; do
    L=exp/lib$X.so; [ "$X" = default ] && L=""
    XP=""
    if [ "${X#p:}" != "$X" ]; then XP=${X#p:}; L=""; X=$(echo "$XP" | tr '=,' '__'); fi
    export EXP_PARAMS=$XP
    D=$O/$X.$n
    GOSSIP_LIB=$L EXP_N=$n EXP_STEPS=${STEPS:-4} timeout -k 10 300 python -u tools/exp_bench.py > $D.txt 2>&1
    ok $? "bench $X $n"
    echo "== $X n=$n: $(tail -1 $D.txt)"
    if [ "${KPROF:-1}" = 1 ]; then
      GOSSIP_LIB=$L EXP_N=$n EXP_STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $D.prof -o run -- python tools/exp_bench.py > $D.prof.txt 2>&1; ok $? "kprof $X $n"
      python tools/kstats.py $(find $D.prof -name '*kernel_stats.csv' | head -1) bin_ frontier_ transpose > $D.kstats
      cat $D.kstats
      python tools/rounds.py $(find $D.prof -name '*kernel_trace.csv' | head -1) > $D.rounds; ok $? rounds
      tail -17 $D.rounds
    fi
    if [ "${PMC:-0}" = 1 ]; then
      i=0
      for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
                 "TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum"; do
        i=$((i+1))
        GOSSIP_LIB=$L EXP_N=$n EXP_STEPS=2 EXP_PARAMS=place_tries=1${XP:+,$XP} timeout -s KILL 120 rocprofv3 --pmc $grp \
          --kernel-trace --output-format csv -d $D.pmc/p$i -o p -- python tools/exp_bench.py > $D.pmc.p$i.txt 2>&1
        ok $? "pmc pass $i $X $n"
      done
      python tools/pmc_dense.py $D.pmc "exp_bench $X n=$n" $D.pmc_dense.json > /dev/null; ok $? pmc_dense
      python tools/pmc_sq.py $D.pmc $D.pmc_sq.json > /dev/null; ok $? pmc_sq
      python -c "
import json; d=json.load(open('$D.pmc_dense.json')); print('$X n=$n PMC:', json.dumps({k: d[k] for k in d if 'round' in k or 'per_node' in k})[:400])"
    fi
  done
done
echo done
