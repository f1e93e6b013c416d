"""Timing experiments: fixed rounds of the dense pipeline (no convergence needed)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import FLAG_DENSE, FLAG_TIMING, Engine
e = Engine(1 << 24, 64, "pushpull", 2, 0x5EED0003, flags=FLAG_DENSE | FLAG_TIMING)
e.inject_random()
e.step(10)  # into the dense middle
for _ in range(3):
    e.step(1)
