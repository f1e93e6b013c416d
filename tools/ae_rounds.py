"""Per-round ANTIENTROPY profile at configs[4] scale (SURVEY.md §8(d) cfg 5: 2^26 nodes, K = 16,
k = 1, churn 1 % / 10 %): round t's device time (timer 0 = churn + round kernels, timer 1 = stats),
its path (dense / sparse), alive nodes and alive-but-stale nodes (alive - full).
The summary gives node-updates/s over the whole run and the roofline fraction of the dense rounds
at 4K(2+2k) = 256 B per node-round (sparse rounds move far fewer bytes, so no fraction is quoted
for them)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import FLAG_TIMING, Engine, loss_threshold
from gossip_hip import engine as _eng
if os.environ.get("GOSSIP_LIB"):  # a library variant (tools/build_variants.sh)
    _eng.load_library(os.environ["GOSSIP_LIB"])
LG = int(sys.argv[1]) if len(sys.argv) > 1 else 26
N, K, k = 1 << LG, 16, 1
HASH = os.environ.get("AE_HASH", "1") != "0"  # AE_HASH=0: no per-round state hash (the reference has none)
# AE_DBIN=0: dense rounds as pull + atomicMax push + stats passes (the round-2 kernels)
e = Engine(N, K, "antientropy", k, 0x5EED0005, flags=(1 if HASH else 0) | FLAG_TIMING,
           churn_fail=loss_threshold(0.01), churn_recover=loss_threshold(0.1),
           params={"ae_dense_bin": int(os.environ.get("AE_DBIN", "1"))})
e.reset(); e.inject_random(); e.step(200)          # warm-up run (first-touch, code load)
e.reset(); e.inject_random(); e.reset_timing()
p0 = p1 = p2 = 0.0
per = {"dense": [], "sparse": []}
prev_stale = None
t0 = time.perf_counter()
for t in range(400):
    r = e.step(1)
    s = r.stats[-1]
    m0, _ = e.kernel_time(0); m1, _ = e.kernel_time(1); m2, _ = e.kernel_time(2)
    d0, d1, d2 = m0 - p0, m1 - p1, m2 - p2
    p0, p1, p2 = m0, m1, m2
    kind = "sparse" if d2 > 0 and d0 == 0 else "dense"  # timer 2: sparse kernels, timer 0: dense
    d0 += d2
    per[kind].append(d0 + d1)
    print(f"{t:3d} {kind:6s} round {d0:8.3f} ms stats {d1:6.3f} ms alive {s['alive_nodes']} "
          f"stale {s['alive_nodes'] - s['full_nodes']} messages {s['messages']}", flush=True)
    if r.converged:
        break
wall = time.perf_counter() - t0
rounds = t + 1
dev = sum(per["dense"]) + sum(per["sparse"])
bpn = 4 * K * (2 + 2 * k)
dn = per["dense"]
print(f"N=2^{LG} K={K} k={k} hash={int(HASH)}: {rounds} rounds to converge, device time {dev:.1f} ms "
      f"(wall {wall * 1e3:.1f} ms incl. per-round host reads)")
print(f"  dense  rounds: {len(dn)}, {sum(dn) / max(len(dn), 1):.3f} ms each, roofline frac "
      f"{bpn * N / (sum(dn) / max(len(dn), 1) * 1e-3) / 8e12:.3f} at {bpn} B per node-round")
sp = per["sparse"]
print(f"  sparse rounds: {len(sp)}, {sum(sp) / max(len(sp), 1):.3f} ms each")
print(f"  node-updates/s: {N * rounds / (dev * 1e-3):.3e} (device time), {N * rounds / wall:.3e} (wall)")
