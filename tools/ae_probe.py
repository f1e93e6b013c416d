"""ANTIENTROPY at configs[4] scale (SURVEY.md §8(d) cfg 5): 2^26 nodes, K = 16 versions,
k = 1, churn p_fail = 0.01, p_recover = 0.1.  Rounds to converge, per-round kernel times
(timer 0 = copy + round kernel, timer 1 = stats), node-updates/s and the roofline
fraction at 4K(2+2k) B per node-round."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import FLAG_TIMING, Engine, loss_threshold
LG = int(sys.argv[1]) if len(sys.argv) > 1 else 26
N, K = 1 << LG, 16
e = Engine(N, K, "antientropy", 1, 0x5EED0005, flags=1 | FLAG_TIMING,
           churn_fail=loss_threshold(0.01), churn_recover=loss_threshold(0.1))
for rep in range(2):
    e.reset(); e.inject_random(); e.reset_timing()
    t0 = time.perf_counter()
    r = e.step(200)
    dt = time.perf_counter() - t0
ms0, n0 = e.kernel_time(0)
ms1, n1 = e.kernel_time(1)
bpn = 4 * K * (2 + 2 * 1)
per_round = (ms0 + ms1) / max(n0, 1)
print(f"N=2^{LG} K={K} rounds={r.rounds} converged={r.converged} wall {dt*1e3:.1f} ms "
      f"round {ms0/max(n0,1):.3f} ms + stats {ms1/max(n1,1):.3f} ms; "
      f"{N * r.rounds / dt:.3e} node-updates/s; roofline {bpn * N / (per_round * 1e-3) / 8e12:.3f}", flush=True)
