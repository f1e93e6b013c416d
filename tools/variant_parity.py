"""Parity of a library variant (GOSSIP_LIB=exp/lib<X>.so, tools/build_variants.sh) against the
OpenMP oracle on one workload: per-round stats, per-rumor counts and the final state, bit for bit.
Usage: GOSSIP_LIB=exp/libX.so python tools/variant_parity.py [log2 nodes] [seed] ["name=value ..."]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import oracle_py as op  # noqa: E402
from gossip_hip import Engine  # noqa: E402
from gossip_hip import engine as _eng  # noqa: E402

if os.environ.get("GOSSIP_LIB"):
    _eng.load_library(os.environ["GOSSIP_LIB"])
# argv[1]: log2 of the node count, or the node count itself when > 64 (odd sizes)
N = (1 << int(sys.argv[1]) if int(sys.argv[1]) <= 64 else int(sys.argv[1])) if len(sys.argv) > 1 else 1 << 27
SEED = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0x5EED0004
PARAMS = {a.split("=")[0]: float(a.split("=")[1]) for a in sys.argv[3].split()} if len(sys.argv) > 3 else {}
e = Engine(N, 64, "pushpull", 2, SEED, flags=1, params=PARAMS)
e.inject_random()
got = e.step(64)
full = e.read_shard()
e.close()
o = op.OracleEngine(N, 64, "pushpull", 2, SEED, flags=1, threads=min(16, os.cpu_count() or 1))
o.inject_random()
want = o.step(64)
ok = got.stats == want.stats and np.array_equal(got.infected, want.infected) and np.array_equal(full, o.read_shard())
print(f"{os.environ.get('GOSSIP_LIB', 'default')}: N={N} rounds {got.rounds} parity {'OK' if ok else 'MISMATCH'}")
sys.exit(0 if ok else 1)
