"""Per round of the bench workload (2^24, push-pull k=2, R=64): fraction of nodes that are
empty / partial / full at the start of the round (what an edge filter on the peer's class
could skip in a dense round)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
import numpy as np
from gossip_hip import Engine
e = Engine(1 << 24, 64, "pushpull", 2, 0x5EED0003, flags=1)
e.inject_random()
for t in range(16):
    s = e.read_shard()[0]
    z = float(np.mean(s == 0)); f = float(np.mean(s == np.uint64(0xFFFFFFFFFFFFFFFF)))
    # edges (n, p) of a dense round that carry nothing in either direction:
    # push needs S[n] not subset of S[p]; a cheap class filter: drop push if p full or n empty,
    # drop pull if p empty or n full; a record is dropped when both are dropped
    push_dead = z + f - z * f   # n empty or p full (independent ends)
    pull_dead = z + f - z * f   # p empty or n full
    both = z * z + f * f + 2 * z * f  # (n empty & p empty) | (n full & p full) | mixed empty/full pairs
    print(f"round {t:2d} empty {z:.3f} full {f:.3f} partial {1 - z - f:.3f}  records droppable ~{both:.3f}", flush=True)
    r = e.step(1)
    if r.converged:
        break
