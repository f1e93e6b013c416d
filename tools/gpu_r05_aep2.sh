#!/bin/bash
# ANTIENTROPY placement over the rows only, 12 candidates: AE GPU tests, one logged configs[4]
# line (exp/libplog.so), then four bench lines.  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_aep2}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_antientropy.py tests/test_gpu_ae_sharded.py -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest_ae.txt 2>&1; ok $?; tail -1 $O/pytest_ae.txt
GOSSIP_LIB=exp/libplog.so timeout -k 10 300 python tools/ae_bench_line.py 1 > $O/ae_line_log.jsonl 2> $O/ae_line_log.err; ok $?
grep ae_place $O/ae_line_log.err
for rep in 1 2 3 4; do
  timeout -k 10 300 python tools/ae_bench_line.py 1 >> $O/ae_line.jsonl 2>> $O/ae_line.err; ok $?
done
python - $O/ae_line_log.jsonl $O/ae_line.jsonl <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        d = json.loads(l)
        print("%s ms_to_converge %.2f dense %.1f us sparse %.1f us" % (f.split("/")[-1], d["ms_to_converge"], d["avg_dense_round_us"], d["avg_sparse_round_us"]))
PY
echo done
