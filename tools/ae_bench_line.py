"""bench.py's configs[4] line alone (antientropy_run: reset + random write + rounds to convergence,
3 timed runs after 1 warm-up), printed as JSON.  Usage: ae_bench_line.py [repeats]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

if os.environ.get("GOSSIP_LIB"):  # a library variant (tools/build_variants.sh)
    from gossip_hip import engine as _eng
    _eng.load_library(os.environ["GOSSIP_LIB"])

for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1):
    print(json.dumps(bench.antientropy_run(0, 3, 1)), flush=True)
