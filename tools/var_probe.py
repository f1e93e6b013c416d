"""Run-to-run variance of the dense round at 2^27 (bench workload, seed of configs[3]): per-step
dense-round averages within one process.  Run it as several processes to separate in-process
(clock, thermal) from per-process (allocation placement) variation.  Not product code."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import FLAG_TIMING, Engine  # noqa: E402
from gossip_hip import engine as _eng  # noqa: E402

if os.environ.get("GOSSIP_LIB"):  # a library variant (tools/build_variants.sh)
    _eng.load_library(os.environ["GOSSIP_LIB"])

N = int(os.environ.get("EXP_N", 1 << 27))
if os.environ.get("DUMMY_MB"):  # device memory held before the engine allocates (placement probe)
    import torch
    hold = torch.empty(int(os.environ["DUMMY_MB"]) << 20, dtype=torch.uint8, device="cuda")
e = Engine(N, 64, "pushpull", 2, 0x5EED0004, flags=FLAG_TIMING)
out = []
for i in range(int(os.environ.get("EXP_STEPS", 6))):
    e.reset_timing()
    e.reset()
    e.inject_random()
    e.step(64, with_infected=False)
    ms, n = e.kernel_time(3)
    out.append(round(ms * 1e3 / max(n, 1), 1))
print(f"{os.environ.get('GOSSIP_LIB', 'default')} dummy {os.environ.get('DUMMY_MB', 0)} MB: dense round us per step:", out[1:])
