"""Parity of an exchange-round library variant (GOSSIP_LIB=exp/lib<X>.so): G shard engines in
lockstep, every dense round an exchange round, against one engine of the same library."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
import numpy as np  # noqa: E402
from gossip_hip import Engine  # noqa: E402
from gossip_hip import engine as _eng  # noqa: E402
from gossip_hip.sharded import lockstep_run  # noqa: E402

if os.environ.get("GOSSIP_LIB"):
    _eng.load_library(os.environ["GOSSIP_LIB"])
for N, G, k in ((1 << 20, 4, 2), (300001, 3, 3), (1 << 22, 8, 1)):
    ref = Engine(N, 64, "pushpull", k, 0x5EED0004, flags=1)
    ref.inject_random()
    want = ref.step(100)
    full = ref.read_shard()
    ref.close()
    es = [Engine(N, 64, "pushpull", k, 0x5EED0004, flags=1, shard_rank=r, shard_count=G,
                 params={"sparse_frac": -1, "xd_shards": 2}) for r in range(G)]
    for e in es:
        e.inject_random()
    got, kinds = lockstep_run(es, 100)
    ok = got == want.stats and set(kinds) == {3} and all(np.array_equal(e.read_shard(), full[:, e.lo:e.hi]) for e in es)
    for e in es:
        e.close()
    print(f"N={N} G={G} k={k}: {'ok' if ok else 'MISMATCH'}", flush=True)
    if not ok:
        sys.exit(1)
