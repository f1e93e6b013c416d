"""One-GPU bench workload (configs[2]: 2^24 nodes, push-pull k=2, 64 rumors; SWEEP_N=134217728 with
seed 0x5EED0004: configs[3]) under gossip_set_param knob sets: ms per step (hipEvents around each
step, timer 0) and rounds.
Usage: sweep_single.py "name=value ..." ["name=value ..." ...]   ("-" = defaults)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import FLAG_TIMING, Engine  # noqa: E402

for spec in sys.argv[1:]:
    params = {} if spec == "-" else {a.split("=")[0]: float(a.split("=")[1]) for a in spec.split()}
    n = int(os.environ.get("SWEEP_N", 1 << 24))
    e = Engine(n, 64, "pushpull", 2, 0x5EED0003 if n == 1 << 24 else 0x5EED0004, flags=FLAG_TIMING, params=params)
    steps = int(os.environ.get("SWEEP_STEPS", 10))
    for i in range(steps + 2):
        if i == 2:
            e.reset_timing()
        e.reset()
        e.inject_random()
        r = e.step(64, with_infected=False)
    ms, n = e.kernel_time(0)
    d, nd = e.kernel_time(3)
    sp, ns = e.kernel_time(4)
    print(f"[{spec}] {ms / steps:.3f} ms/step, rounds {r.rounds}, dense rounds/step {nd / steps:.1f}, "
          f"dense {d * 1e3 / max(nd, 1):.1f} us, sparse {sp / steps:.3f} ms/step in {ns / steps:.1f} rounds", flush=True)
    e.close()
