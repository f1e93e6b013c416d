#!/bin/bash
# Placement calibration at its default (place_tries 8): parity of the dense paths, 4 processes of
# tools/place_probe4.py, then the bench line (configs[3], with configs[2] and configs[4]).
set -u
O=gpurun_out/${1:-r05_pl7}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cfg4_full.py::test_cfg4_single_engine_equals_oracle tests/test_gpu_big_paths.py -m gpu -q --timeout 300 --timeout-method thread -x > $O/pytest.txt 2>&1 || { echo STOP tests; tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for rep in 1 2 3 4; do
  timeout -k 10 150 python tools/place_probe4.py >> $O/probe.txt 2>&1 || { echo "STOP"; tail -5 $O/probe.txt; exit 1; }
  tail -1 $O/probe.txt
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo STOP bench; tail -5 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]; s = d["secondary"]; a = d["antientropy"]
print("2^27 %.3g nu/s %.2f ms/step dense %.0f us frac %.3f sparse %.0f us | 2^24 %.3g dense %.0f sparse %.0f | AE %.1f ms" % (d["value"], d["ms_per_step"], r["avg_launch_us"], r["frac"], r["sparse_rounds"]["avg_round_us"], s["value"], s["avg_dense_round_us"], s["sparse_avg_round_us"], a["ms_to_converge"]))
PY
