"""Placement probe 3: one 2^27 engine (an experiment build with GOSSIP_EXP_REALLOC, GOSSIP_LIB=...);
its dense-round time (bench workload, timer 3), then again after each fresh allocation of the
buffers named by PROBE_MASK (1 the bin slab, 2 the state image, 4 the frontier buffers), the old
ones kept.  Shows which allocation carries the fast / slow mode.  Not product code; the
exp_realloc param it sets existed only in that experiment build and was removed once
profiles/r05_pl/r05_pl4/ had answered (the record slab; engine.hip place_bins)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import FLAG_TIMING, Engine  # noqa: E402
from gossip_hip import engine as _eng  # noqa: E402

_eng.load_library(os.environ["GOSSIP_LIB"])
e = Engine(1 << 27, 64, "pushpull", 2, 0x5EED0004, flags=FLAG_TIMING)


def dense_us(steps=2):
    out = []
    for i in range(steps + 1):
        e.reset_timing()
        e.reset()
        e.inject_random()
        e.step(64, with_infected=False)
        ms, n = e.kernel_time(3)
        out.append(round(ms * 1e3 / max(n, 1), 1))
    return out[1:]


mask = int(os.environ.get("PROBE_MASK", 1))
print(f"mask {mask} initial: {dense_us()}", flush=True)
for i in range(int(os.environ.get("PROBE_TRIES", 6))):
    e.set_param("exp_realloc", mask)
    print(f"mask {mask} realloc {i}: {dense_us()}", flush=True)
