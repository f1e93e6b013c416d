#!/bin/bash
# Round 5: ANTIENTROPY with the lazy zeroing after reset and one read-back per round: the AE GPU
# tests, then bench.py's configs[4] line three times (tools/ae_bench_line.py).  Output under gpurun_out/$1.
set -u
O=gpurun_out/${1:-r05_ae4}
mkdir -p $O
export TMPDIR=/tmp
ok() { local rc=$1; if [ "$rc" -ne 0 ]; then echo "STOP: step exited $rc"; exit "$rc"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_antientropy.py tests/test_gpu_ae_sharded.py -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest_ae.txt 2>&1; ok $?; tail -1 $O/pytest_ae.txt
timeout -k 10 400 python tools/ae_bench_line.py 3 > $O/ae_line.jsonl 2> $O/ae_line.err; ok $?
python - $O/ae_line.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print("ms_to_converge %.2f rounds %d dense %.1f us sparse %.1f us" % (d["ms_to_converge"], d["rounds_to_converge"], d["avg_dense_round_us"], d["avg_sparse_round_us"]))
PY
echo done
