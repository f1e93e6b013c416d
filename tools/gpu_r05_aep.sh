#!/bin/bash
# ANTIENTROPY placement calibration (ae_place): the AE GPU tests, one configs[4] line with each
# candidate's trial logged (exp/libplog.so), then bench.py's configs[4] line three times.
set -u
O=gpurun_out/${1:-r05_aep}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_antientropy.py tests/test_gpu_ae_sharded.py -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest_ae.txt 2>&1; ok $?; tail -1 $O/pytest_ae.txt
GOSSIP_LIB=exp/libplog.so timeout -k 10 300 python tools/ae_bench_line.py 1 > $O/ae_line_log.jsonl 2> $O/ae_line_log.err; ok $?
grep ae_place $O/ae_line_log.err
timeout -k 10 400 python tools/ae_bench_line.py 3 > $O/ae_line.jsonl 2> $O/ae_line.err; ok $?
python - $O/ae_line_log.jsonl $O/ae_line.jsonl <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        d = json.loads(l)
        print("%s ms_to_converge %.2f rounds %d dense %.1f us sparse %.1f us" % (f.split("/")[-1], d["ms_to_converge"], d["rounds_to_converge"], d["avg_dense_round_us"], d["avg_sparse_round_us"]))
PY
echo done
