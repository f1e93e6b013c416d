"""Placement calibration check: one 2^27 (PROBE_N) engine per process with param place_tries = PROBE_TRIES
(1: the first allocation of the record slab; n: the fastest of n zero-state trial rounds; unset:
the default),
its dense-round time on the bench workload (timer 3) and its trial rounds (timer 5).  Not product code."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import FLAG_TIMING, Engine  # noqa: E402
from gossip_hip import engine as _eng  # noqa: E402

if os.environ.get("GOSSIP_LIB"):  # a library variant (tools/build_variants.sh)
    _eng.load_library(os.environ["GOSSIP_LIB"])

tries = os.environ.get("PROBE_TRIES")  # unset: the engine's default
N = int(os.environ.get("PROBE_N", 1 << 27))
e = Engine(N, 64, "pushpull", 2, 0x5EED0004 if N == 1 << 27 else 0x5EED0003, flags=FLAG_TIMING,
           params={"place_tries": int(tries)} if tries else {})
out = []
trial = None
for i in range(4):
    if i == 1:
        trial = e.kernel_time(5)
    e.reset_timing()
    e.reset()
    e.inject_random()
    e.step(64, with_infected=False)
    ms, n = e.kernel_time(3)
    out.append(round(ms * 1e3 / max(n, 1), 1))
print(f"place_tries {tries}: trial rounds {trial[1]} avg {trial[0] * 1e3 / max(trial[1], 1):.1f} us; "
      f"dense round us {out[1:]}", flush=True)
