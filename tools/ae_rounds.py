"""Per-round ANTIENTROPY profile at configs[4] scale: round t's kernel time (timer 0 = seed copy +
round kernel, timer 1 = stats), alive nodes and alive-but-stale nodes (alive - full)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import FLAG_TIMING, Engine, loss_threshold
LG = int(sys.argv[1]) if len(sys.argv) > 1 else 26
N, K = 1 << LG, 16
e = Engine(N, K, "antientropy", 1, 0x5EED0005, flags=1 | FLAG_TIMING,
           churn_fail=loss_threshold(0.01), churn_recover=loss_threshold(0.1))
e.reset(); e.inject_random(); e.reset_timing()
p0 = p1 = 0.0
tot = 0.0
for t in range(200):
    r = e.step(1)
    s = r.stats[-1]
    m0, _ = e.kernel_time(0); m1, _ = e.kernel_time(1)
    d0, d1 = m0 - p0, m1 - p1
    p0, p1 = m0, m1
    tot += d0 + d1
    print(f"{t:3d} round {d0:8.3f} ms stats {d1:6.3f} ms alive {s['alive_nodes']} stale {s['alive_nodes'] - s['full_nodes']}", flush=True)
    if r.converged:
        break
print(f"total {tot:.1f} ms over {t + 1} rounds")
