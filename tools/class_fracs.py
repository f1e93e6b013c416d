"""Per-round class fractions of the bench workload (one engine, one round per step call): nonzero
and full nodes after each round, the rare fraction the planner sees, and the share of peers that
would hit the LDS summary (1 - (1 - r)^g) — the input of the mid-level summary threshold
(mid_frac).  Usage: class_fracs.py [log2 nodes]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import Engine  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 27
N = 1 << lg
e = Engine(N, 64, "pushpull", 2, 0x5EED0004 if lg == 27 else 0x5EED0003)
e.inject_random()
g = 1
while (N + g - 1) // g > (1 << 20):
    g *= 2
for t in range(20):
    s = e.read_shard().ravel()  # (one engine: the totals are internal; the state is 8 B per node)
    full, nz = int((s == (2 ** 64 - 1)).sum()), int((s != 0).sum())
    r = min(nz, N - full) / N
    print(f"before round {t:2d}: nonzero {nz / N:.5f} full {full / N:.5f} rare {r:.5f} lds_hit {1 - (1 - r) ** g:.3f} "
          f"mid_hit {1 - (1 - r) ** 8:.3f}", flush=True)
    res = e.step(1, with_infected=False)
    if res.converged:
        break
