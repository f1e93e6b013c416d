"""FLOOD (the reference's own rule, main.go:65-89) at scale: a random directed topology with d
out-neighbours per node (Maelstrom hands the reference arbitrary topologies; a random one keeps
the diameter small), 64 rumors at Philox origins, rounds until quiescent.  Prints rounds,
messages (RPCs the reference would send) and device time per round (timer 0).
Usage: flood_probe.py [log2 N] [d]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
import numpy as np  # noqa: E402
from gossip_hip import FLAG_TIMING, Engine  # noqa: E402

LG = int(sys.argv[1]) if len(sys.argv) > 1 else 22
D = int(sys.argv[2]) if len(sys.argv) > 2 else 8
N = 1 << LG
rng = np.random.default_rng(7)
col = rng.integers(0, N - 1, size=N * D, dtype=np.uint64).astype(np.uint32)
own = np.repeat(np.arange(N, dtype=np.uint32), D)
col = np.where(col >= own, col + 1, col).astype(np.uint32)  # no self loops
row_ptr = (np.arange(N + 1, dtype=np.uint64) * D).astype(np.uint32)
e = Engine(N, 64, "flood", 1, 0x5EED0007, flags=FLAG_TIMING)
t0 = time.perf_counter()
e.set_topology((row_ptr, col))
print(f"N=2^{LG} d={D}: topology of {N * D} edges set in {time.perf_counter() - t0:.1f} s", flush=True)
for rep in range(3):
    if rep == 1:
        e.reset_timing()
    e.reset()
    e.inject_random()
    res = e.step(256, with_infected=False)
ms, n = e.kernel_time(0)
msgs = sum(s["messages"] for s in res.stats)
edges = N * D
per_round = ms / max(n, 1)
print(f"rounds {res.rounds}, messages {msgs}, full after {res.stats[-1]['full_nodes']} of {N}; "
      f"{per_round * 1e3:.1f} us per round, {edges / (per_round / 1e3) / 1e9:.1f} G edge-visits/s, "
      f"{N / (per_round / 1e3) / 1e9:.1f} G node-updates/s", flush=True)
