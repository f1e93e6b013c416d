"""configs[4] (2^26 nodes, K = 16, k = 1, churn 1 % / 10 %, seed 0x5EED0005) to convergence in one
gossip_step, as bench.py's `antientropy` line runs it: wall time per run, rounds, dense / sparse
device time.  AE_AHEAD: the engine's ae_ahead (pipelined sparse rounds, engine step_ae); AE_TIMING=0
drops the per-round events.  Reference: main.go:77-87 (retry until acked), DESIGN.md §3.8."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
import torch  # noqa: E402,F401  (the HIP runtime, as bench.py has it)
from gossip_hip import FLAG_TIMING, Engine, loss_threshold  # noqa: E402
from gossip_hip import engine as _eng  # noqa: E402

if os.environ.get("GOSSIP_LIB"):  # a variant build (tools/build_variants.sh)
    _eng.load_library(os.environ["GOSSIP_LIB"])

N, K, k, seed = 1 << int(os.environ.get("AE_LG", 26)), 16, 1, 0x5EED0005
timing = os.environ.get("AE_TIMING", "1") != "0"
e = Engine(N, K, "antientropy", k, seed, flags=FLAG_TIMING if timing else 0,
           churn_fail=loss_threshold(0.01), churn_recover=loss_threshold(0.1),
           params={"ae_ahead": int(os.environ.get("AE_AHEAD", 8)),
                   # AE_PARAMS="name=value,...": more gossip_set_param knobs (e.g. ae_dense_filter=0)
                   **{kv.split("=")[0]: float(kv.split("=")[1]) for kv in os.environ.get("AE_PARAMS", "").split(",") if kv}})
runs = int(os.environ.get("AE_RUNS", 3))
for i in range(runs + 1):
    if i == 1:
        e.reset_timing()
        t0 = time.perf_counter()
    e.reset()
    e.inject_random()
    r = e.step(400, with_infected=False)
    assert r.converged
wall = (time.perf_counter() - t0) / runs
d, dn = e.kernel_time(0)
s, sn = e.kernel_time(2)
st, _ = e.kernel_time(1)
print(f"{os.environ.get('GOSSIP_LIB', 'default')} {os.environ.get('AE_PARAMS', '')} ae_ahead={os.environ.get('AE_AHEAD', 8)} timing={int(timing)}: {r.rounds} rounds, wall {wall * 1e3:.1f} ms per run, "
      f"dense {dn // runs} x {d / max(dn, 1):.3f} ms, sparse {sn // runs} x {s / max(sn, 1):.3f} ms, "
      f"device {(d + s + st) / runs:.1f} ms per run, {N * r.rounds / wall:.3e} node-updates/s")
