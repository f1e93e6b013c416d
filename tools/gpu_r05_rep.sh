#!/bin/bash
# Repeat bench lines (separate processes, no tests) for the run-to-run spread of the final tree.
set -u
O=gpurun_out/${1:-r05_rep}
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_rep$rep.json 2> $O/bench_rep$rep.err || { echo STOP; tail -5 $O/bench_rep$rep.err; exit 1; }
  python - $O/bench_rep$rep.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]; s = d["secondary"]; a = d["antientropy"]
print("%.4g nu/s %.2f ms/step dense %.0f us frac %.3f sparse %.0f | 2^24 %.4g dense %.0f sparse %.0f | AE %.1f ms | verified %s" % (d["value"], d["ms_per_step"], r["avg_launch_us"], r["frac"], r["sparse_rounds"]["avg_round_us"], s["value"], s["avg_dense_round_us"], s["sparse_avg_round_us"], a["ms_to_converge"], d["verified"]))
PY
done
