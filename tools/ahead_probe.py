"""ms per bench step vs run-ahead depth and hipEvent timing (configs[2] workload)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
import torch
from gossip_hip import FLAG_TIMING, Engine
for ahead in (1, 2, 3, 4, 6):
    for timing in (0, FLAG_TIMING):
        os.environ["GOSSIP_AHEAD"] = str(ahead)
        e = Engine(1 << 24, 64, "pushpull", 2, 0x5EED0003, flags=timing)
        def step():
            e.reset(); e.inject_random(); return e.step(64).rounds
        step(); step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5): r = step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        print(f"ahead {ahead} timing {bool(timing)}: {dt*1e3:.3f} ms/step rounds {r}", flush=True)
        e.close()
