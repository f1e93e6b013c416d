"""Placement probe 2: one 2^27 engine per process, optionally after a large device allocation was
made and released to the driver first (PROBE_PRE_GB; hipMalloc + hipFree through torch with
empty_cache), or while one is held (PROBE_HOLD_GB).  Prints the dense-round time (bench workload, timer 3).  Not product code."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
import torch  # noqa: E402
from gossip_hip import FLAG_TIMING, Engine  # noqa: E402

pre = int(os.environ.get("PROBE_PRE_GB", 0))
if pre:
    x = torch.empty(pre << 30, dtype=torch.uint8, device="cuda")
    del x
    torch.cuda.empty_cache()
hold_gb = int(os.environ.get("PROBE_HOLD_GB", 0))  # device memory held while the engine allocates
hold = torch.empty(hold_gb << 30, dtype=torch.uint8, device="cuda") if hold_gb else None
e = Engine(1 << 27, 64, "pushpull", 2, 0x5EED0004, flags=FLAG_TIMING)
out = []
for i in range(4):
    e.reset_timing()
    e.reset()
    e.inject_random()
    e.step(64, with_infected=False)
    ms, n = e.kernel_time(3)
    out.append(round(ms * 1e3 / max(n, 1), 1))
print(f"pre {pre} GB hold {hold_gb} GB: dense round us {out[1:]}", flush=True)
