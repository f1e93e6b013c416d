"""Timing experiments on the dense pipeline.

Default: FLAG_DENSE, 10 rounds into the dense middle, then 3 single rounds.
EXP_AUTO=1: the normal path choice; rounds 0-6 run on the sparse path (identical
in every dense-kernel variant), so round 7 — the first dense round — starts
from the same state in every variant and its kernel times compare directly.
"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import FLAG_DENSE, FLAG_TIMING, Engine
from gossip_hip import engine as _eng
if os.environ.get("GOSSIP_LIB"):  # experiment variant of the library (tools/gpu_variants.sh)
    _eng.load_library(os.environ["GOSSIP_LIB"])
auto = os.environ.get("EXP_AUTO") == "1"
e = Engine(1 << 24, 64, "pushpull", 2, 0x5EED0003, flags=FLAG_TIMING | (0 if auto else FLAG_DENSE))
for rep in range(3 if auto else 1):
    e.reset()
    e.inject_random()
    e.step(int(os.environ.get("EXP_BEFORE", "7")) if auto else 10)
    for _ in range(1 if auto else 3):
        e.step(1)
