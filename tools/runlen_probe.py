"""Dense binned pipeline cost per node-round vs N (run length = ts*k / nt_d records)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
from gossip_hip import FLAG_DENSE, FLAG_TIMING, Engine
for lg in (21, 22, 23, 24, 25, 26):
    N = 1 << lg
    e = Engine(N, 64, "pushpull", 2, 0x5EED0003, flags=FLAG_DENSE | FLAG_TIMING)
    for rep in range(2):
        e.reset(); e.inject_random(); e.reset_timing()
        r = e.step(64)
    ms, n = e.kernel_time(0)
    runlen = 16384 / max(1, N // 16384)
    print(f"N=2^{lg} runlen={runlen:.0f} rounds={r.rounds} us/round={ms*1e3/n:.1f} ns/node-round={ms*1e6/n/N:.3f}", flush=True)
    e.close()
