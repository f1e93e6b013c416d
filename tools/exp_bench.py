"""The bench workload (configs[2]: 2^24 nodes, push-pull k=2, 64 rumors) on a library variant
(GOSSIP_LIB=exp/lib<X>.so, tools/build_variants.sh), for per-kernel timing under rocprofv3:
tools/rounds.py then splits the trace into rounds.  Prints the dense-round average (timer 3)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import FLAG_TIMING, Engine  # noqa: E402
from gossip_hip import engine as _eng  # noqa: E402

if os.environ.get("GOSSIP_LIB"):
    _eng.load_library(os.environ["GOSSIP_LIB"])
N = int(os.environ.get("EXP_N", 1 << 24))
# EXP_PARAMS="name=value,...": gossip_set_param knobs (e.g. fuse_emit=0)
PARAMS = {kv.split("=")[0]: float(kv.split("=")[1]) for kv in os.environ.get("EXP_PARAMS", "").split(",") if kv}
e = Engine(N, 64, "pushpull", 2, int(os.environ.get("EXP_SEED", "0x5EED0003"), 0), flags=FLAG_TIMING, params=PARAMS)
for i in range(int(os.environ.get("EXP_STEPS", 4))):
    if i == 1:
        e.reset_timing()
    e.reset()
    e.inject_random()
    r = e.step(64, with_infected=False)
ms, n = e.kernel_time(3)
sms, sn = e.kernel_time(4)
tms, tn = e.kernel_time(0)
steps = int(os.environ.get("EXP_STEPS", 4)) - 1
print(f"{os.environ.get('GOSSIP_LIB', 'default')}: rounds {r.rounds}, dense rounds {n}, "
      f"{ms * 1e3 / max(n, 1):.1f} us per dense round, sparse {sms * 1e3 / max(sn, 1):.1f} us per round, "
      f"step {tms / max(steps, 1):.3f} ms of device time")
