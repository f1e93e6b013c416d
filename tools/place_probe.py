"""Is the dense round's fast / slow placement mode (DESIGN.md §3.7 'bimodal across processes') a
property of the process or of each allocation?  Creates several 2^27 engines in one process, all
kept alive, and prints each one's dense-round time (bench workload, timer 3); then frees them
and creates two more.  Not product code."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import FLAG_TIMING, Engine  # noqa: E402


def dense_us(e, steps=3):
    out = []
    for i in range(steps + 1):
        e.reset_timing()
        e.reset()
        e.inject_random()
        e.step(64, with_infected=False)
        ms, n = e.kernel_time(3)
        out.append(round(ms * 1e3 / max(n, 1), 1))
    return out[1:]


N = 1 << 27
keep = []
for i in range(int(os.environ.get("PROBE_ENGINES", 5))):
    e = Engine(N, 64, "pushpull", 2, 0x5EED0004, flags=FLAG_TIMING)
    keep.append(e)
    print(f"engine {i} (kept): dense round us {dense_us(e)}", flush=True)
print(f"engine 0 again: dense round us {dense_us(keep[0])}", flush=True)
for e in keep:
    e.close()
keep.clear()
for i in range(2):
    e = Engine(N, 64, "pushpull", 2, 0x5EED0004, flags=FLAG_TIMING)
    print(f"after free, engine {i}: dense round us {dense_us(e)}", flush=True)
    e.close()
