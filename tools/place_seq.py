"""Placement calibration over engines made one after another in one process:
PROBE_ENGINES engines of PROBE_N nodes (bench workload: configs[3] at 2^27, configs[2] at 2^24),
each created, run for 4 steps (the first carries the placement trials) and closed before the next.
Per engine: the dense-round time of steps 2-4 (timer 3), the trial rounds (timer 5), the first
step's wall time against a later step's (what the trials add to the first gossip_step), and the
device memory in use around the first step (torch.cuda.mem_get_info; the trials' transient peak is
bounded by construction: the kept slab plus two).  Not product code."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
import torch  # noqa: E402
from gossip_hip import FLAG_TIMING, Engine  # noqa: E402
from gossip_hip import engine as _eng  # noqa: E402

if os.environ.get("GOSSIP_LIB"):
    _eng.load_library(os.environ["GOSSIP_LIB"])
N = int(os.environ.get("PROBE_N", 1 << 27))
seed = 0x5EED0004 if N == 1 << 27 else 0x5EED0003
tries = os.environ.get("PROBE_TRIES")
res = []
for i in range(int(os.environ.get("PROBE_ENGINES", 4))):
    e = Engine(N, 64, "pushpull", 2, seed, flags=FLAG_TIMING, params={"place_tries": int(tries)} if tries else {})
    walls, dense = [], []
    free0 = torch.cuda.mem_get_info()[0]
    low = [free0]
    for s in range(4):
        e.reset_timing()
        e.reset()
        e.inject_random()
        stop = threading.Event()

        def sample():  # the least free device memory while the first step (and its trials) runs
            while not stop.is_set():
                low[0] = min(low[0], torch.cuda.mem_get_info()[0])
                time.sleep(0.002)
        th = threading.Thread(target=sample) if s == 0 and not os.environ.get("PROBE_NOSAMPLE") else None
        if th:
            th.start()
        t0 = time.perf_counter()
        e.step(64, with_infected=False)
        walls.append((time.perf_counter() - t0) * 1e3)
        if th:
            stop.set()
            th.join()
        if s == 0:
            trial = e.kernel_time(5)
        ms, n = e.kernel_time(3)
        dense.append(ms * 1e3 / max(n, 1))
    free1 = torch.cuda.mem_get_info()[0]
    e.close()
    d = sorted(dense[1:])
    res.append(d[1])
    print(f"engine {i}: dense round us {[round(x, 1) for x in dense[1:]]}, trial rounds {trial[1]} "
          f"({trial[0]:.1f} ms of device time), first step {walls[0]:.1f} ms vs {min(walls[1:]):.1f} ms, "
          f"peak extra device memory during the first step {(free0 - low[0]) / 2**30:.2f} GiB "
          f"(after it {(free0 - free1) / 2**30:.2f} GiB)", flush=True)
print(f"N={N}: median dense round per engine {[round(x, 1) for x in res]} us; "
      f"max {max(res):.1f} us over {len(res)} engines", flush=True)
