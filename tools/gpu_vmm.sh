#!/bin/bash
# Round-6 placement experiment: the record slab from the VMM API (exp/libvmm*.so,
# tools/build_variants.sh with GOSSIP_SLAB_VMM) against hipMalloc with and without the trials, over
# engines made one after another (tools/place_seq.py).  TRIES: place_tries of the exp/ variants
# (default 1).  Every step under its own limit.
set -u
O=gpurun_out/${OUT:-vmm}
mkdir -p $O
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: $2 exited $rc"; exit "$rc"; fi; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; ok $? smoke
tail -1 $O/smoke.txt
for v in ${VARS:-default1 vmm1 vmm2 vmm3 vmm3b default12}; do
  for q in ${SEQ:-134217728:3 16777216:6}; do
    L=exp/lib$v.so; T=${TRIES:-1}
    case $v in default1) L=""; T=1;; default12) L=""; T=12;; esac
    GOSSIP_LIB=$L PROBE_TRIES=$T PROBE_NOSAMPLE=1 PROBE_N=${q%%:*} PROBE_ENGINES=${q##*:} \
      timeout -k 10 300 python -u tools/place_seq.py > $O/seq_${v}_${q%%:*}.txt 2>&1
    ok $? "place_seq $v $q"
    echo "== $v $q"; tail -1 $O/seq_${v}_${q%%:*}.txt
  done
done
