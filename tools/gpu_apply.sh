#!/bin/bash
# Persistent apply A/B: dense-path parity, per-kernel dense-round times for
# one-block-per-tile apply (GOSSIP_APPLY_GRID=0), persistent apply, and the
# prefetch variants exp/libpre{2,4}.so; bench with and without.
set -u
mkdir -p gpurun_out/apply
export TMPDIR=/tmp
O=gpurun_out/apply
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_gpu_faults.py tests/test_gpu_multiprocess.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; echo "STOP tests"; exit 1; }
tail -1 $O/pytest.log
run() {  # name, env...
  local X=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$X -o run -- python tools/exp_rounds.py > $O/$X.out 2>&1 || { echo "STOP $X"; exit 1; }
  echo "== $X"; python tools/rounds.py $O/$X/run_kernel_trace.csv | grep dense | tail -4
}
run tile GOSSIP_APPLY_GRID=0
run pers GOSSIP_APPLY_GRID=256
run pre2 GOSSIP_LIB=exp/libpre2.so
run pre4 GOSSIP_LIB=exp/libpre4.so
for G in 0 256 0 256; do
  GOSSIP_APPLY_GRID=$G timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$G.json 2> $O/bench.err || { echo "STOP bench"; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$G.json')); r=d['roofline']; print('grid $G', round(d['value']/1e9,2), 'G', round(d['ms_per_step'],3), 'ms; dense-only round', round(r['dense_only']['avg_round_us'],1), 'us')"
done
echo done
