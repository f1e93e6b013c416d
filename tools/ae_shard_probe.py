"""Per-rank cost of sharded ANTIENTROPY rounds (configs[4]: 2^26 nodes, K = 16, fanout 1, churn
1 % / 10 %, seed 0x5EED0005) at G shards, all G engines on one GPU in one process
(gossip_hip.sharded lockstep protocol): every engine call of a round is timed
(one rank's device work; collectives excluded) and the bytes a rank receives are recorded (the
stale-word all-gather, request items in, replies back).  The one-GPU engine runs the same
workload for comparison.  usage: python tools/ae_shard_probe.py [G] [log2 N]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gossip_hip import FLAG_TIMING, Engine  # noqa: E402
from gossip_hip import sharded as sh  # noqa: E402
from gossip_hip import engine as _eng  # noqa: E402
from gossip_hip.engine import churn_threshold as ct  # noqa: E402

if os.environ.get("GOSSIP_LIB"):  # a library variant (tools/build_variants.sh)
    _eng.load_library(os.environ["GOSSIP_LIB"])

G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
N = 1 << (int(sys.argv[2]) if len(sys.argv) > 2 else 26)
K, k, seed = 16, 1, 0x5EED0005
kw = dict(churn_fail=ct(0.01), churn_recover=ct(0.1))
CALLS = ("exchange_buffers", "ae_requests", "ae_request_recv", "ae_serve", "ae_response_recv", "ae_finish",
         "ae_local_target", "ae_set_target", "round_commit")


class Timed:
    def __init__(self, e, log):
        self._e, self._log = e, log
        self.recv = 0

    def __getattr__(self, name):
        f = getattr(self._e, name)
        if name not in CALLS:
            return f

        def g(*a):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = f(*a)
            torch.cuda.synchronize()
            self._log.append((name, (time.perf_counter() - t0) * 1e3))
            if name == "exchange_buffers":
                self.recv += (G - 1) * r[2]
            elif name == "ae_requests":  # items out ~ items in (symmetry), request + reply words
                words = self._e.ae_item_words(0) + self._e.ae_item_words(1)
                self.recv += 4 * words * (sum(r[1]) - r[1][self._e.shard_rank_])
            return r
        return g


# one GPU
ref = Engine(N, K, "antientropy", k, seed, flags=FLAG_TIMING, **kw)
for rep in range(2):
    ref.reset()
    ref.inject_random()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = ref.step(400)
    torch.cuda.synchronize()
    one_ms = (time.perf_counter() - t0) * 1e3
print(f"one GPU: N=2^{int(np.log2(N))} {res.rounds} rounds in {one_ms:.1f} ms wall, "
      f"{N * res.rounds / one_ms / 1e6:.3g} G node-updates/s", flush=True)
ref.close()

engines = [Engine(N, K, "antientropy", k, seed, flags=0, shard_rank=r, shard_count=G, **kw) for r in range(G)]
for r, e in enumerate(engines):
    e.shard_rank_ = r
for rep in range(2):
    logs = [[] for _ in engines]
    tes = [Timed(e, lg) for e, lg in zip(engines, logs)]
    for e in engines:
        e.reset()
        e.inject_random()
    rounds = []
    for t in range(400):
        for lg in logs:
            lg.clear()
        for te in tes:
            te.recv = 0
        ks = [e.sharded_plan() for e in engines]
        if ks[0] == -2:
            tgt = np.maximum.reduce([te.ae_local_target() for te in tes])
            for te in tes:
                te.ae_set_target(tgt)
            ks = [e.sharded_plan() for e in engines]
        assert ks[0] == 2, ks
        parts = sh._lockstep_ae(tes)
        tot = sh._lockstep_sum(parts)
        st = [te.round_commit(tot) for te in tes]
        per_rank = np.mean([sum(ms for _, ms in lg) for lg in logs])
        calls = {}
        for lg in logs:
            for name, ms in lg:
                calls[name] = calls.get(name, 0.0) + ms / len(logs)
        rounds.append((t, per_rank, tes[0].recv, int(st[0]["alive_nodes"]), int(st[0]["full_nodes"]), calls))
        if st[0]["converged"]:
            break
    if rep == 1:
        for t, ms, rb, alive, full, calls in rounds:
            if t < 16 or t % 10 == 0 or t == len(rounds) - 1:
                br = " ".join(f"{n}={v:.3f}" for n, v in calls.items()) if t in (0, 50) else ""
                print(f"G={G} round {t:3d} per-rank {ms:7.3f} ms  recv {rb / 2**20:7.1f} MiB  alive={alive} "
                      f"stale={alive - full}  {br}", flush=True)
        tot_ms = sum(r[1] for r in rounds)
        print(f"G={G} N=2^{int(np.log2(N))} rounds={len(rounds)} sum per-rank {tot_ms:.1f} ms  "
              f"recv per rank {sum(r[2] for r in rounds) / 2**20:.1f} MiB  "
              f"{N * len(rounds) / tot_ms / 1e6:.3g} G node-updates/s on per-rank device time", flush=True)
