"""Per-rank cost of sharded rounds at G shards x 2^24 nodes, all G engines on one GPU in
one process (gossip_hip.sharded.lockstep_run): every engine call is timed (that is one
rank's device work), and the bytes each exchange moves per rank are recorded ("gathered":
state all-gathers as received; exchange rounds: the class bitmaps received plus 20 B per item
the rank sends off-rank, its 12-B item out and 8-B reply back, which by symmetry is what it
also receives).  The link
time of a real G-GPU run is not measured here: DESIGN.md §5 prices it."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
import numpy as np
import torch
from gossip_hip import Engine
from gossip_hip import engine as _eng
from gossip_hip import sharded as sh

if os.environ.get("GOSSIP_LIB"):  # a library variant (tools/build_variants.sh)
    _eng.load_library(os.environ["GOSSIP_LIB"])

G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
LG = int(sys.argv[2]) if len(sys.argv) > 2 else 24
CALLS = ("sparse_rare", "sparse_scan", "sparse_commit", "dense_prepare", "round_compute", "exchange_buffers",
         "local_totals", "xd_classes", "xd_requests", "xd_request_recv", "xd_serve", "xd_response_recv", "xd_finish",
         "cc_send", "cc_recv", "cc_expand")
# argv[3:]: gossip_set_param knobs as name=value (e.g. xd_shards=0: dense rounds on the state all-gather)
PARAMS = {a.split("=")[0]: float(a.split("=")[1]) for a in sys.argv[3:]}


class Timed:
    """Times the engine calls of one rank; gathered: state bytes the rank receives this round."""

    def __init__(self, e, log, rank):
        self._e, self._log, self._rank = e, log, rank
        self.gathered = 0

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
                self.gathered = (G - 1) * r[2]
            elif name == "cc_send":
                self.gathered = (G - 1) * r[1]
            elif name == "cc_recv":
                self.gathered += (G - 1) * a[0] * 8
            elif name == "xd_classes":
                self.gathered = (G - 1) * r[2]
            elif name == "xd_requests":  # items in (12 B) and replies in (8 B), ~ the items it sends off-rank
                self.gathered += 20 * (sum(r[2]) - r[2][self._rank])
            elif name == "sparse_rare":  # its rare list to every other rank (16-B items); by symmetry ~ what it receives
                self.gathered = (G - 1) * 16 * r[1]
            elif name == "sparse_scan":  # pushes for other shards (16-B items)
                self.gathered += 16 * (sum(int(c) for c in r[1]) - int(r[1][self._rank]))
            return r
        return g


engines = [Engine(G << LG, 64, "pushpull", 2, 0x5EED0004, shard_rank=r, shard_count=G, params=PARAMS)
           for r in range(G)]
for rep in range(2):
    logs = [[] for _ in engines]
    tes = [Timed(e, l, r) for r, (e, l) in enumerate(zip(engines, logs))]
    for e in engines:
        e.reset(); e.inject_random()
    rounds = []
    for t in range(64):
        for l in logs: l.clear()
        for te in tes: te.gathered = 0
        ks = [e.sharded_plan() for e in engines]
        if ks[0] < 0:
            tot = sh._lockstep_sum([e.local_totals() for e in engines]); ks = [e.sharded_plan(tot) for e in engines]
        if ks[0] == 1:
            parts = sh._lockstep_sparse(tes)
        elif ks[0] == 3:
            parts = sh._lockstep_xd(tes)
        elif ks[0] in (4, 7):  # (7: class-coded all-gather, then the replicated round)
            parts = sh._lockstep_cc(tes)
        elif ks[0] == 6:  # replicated on the whole image: no exchange
            parts = [te.round_compute() for te in tes]
        else:
            parts = sh._lockstep_dense(tes)
        tot = sh._lockstep_sum(parts)
        st = [e.round_commit(tot) for e in engines]
        per_rank = np.mean([sum(ms for _, ms in l) for l in logs])
        calls = {}
        for l in logs:
            for name, ms in l:
                calls[name] = calls.get(name, 0.0) + ms / len(logs)
        rounds.append((t, ks[0], per_rank, int(st[0]["full_nodes"]), calls, tes[0].gathered))
        if st[0]["converged"]:
            break
    if rep == 1:
        for t, k, ms, full, calls, gb in rounds:
            br = " ".join(f"{n}={v:.3f}" for n, v in calls.items())
            kind = ['dense ', 'sparse', 'ae', 'xdense', 'ccoded', 'rep-ag', 'rep   ', 'rep-cc'][k]
            print(f"G={G} round {t:2d} {kind} per-rank {ms:7.3f} ms  full={full}  gathered={gb / 2**20:.1f} MiB  [{br}]",
                  flush=True)
        print(f"G={G} rounds={len(rounds)} sum per-rank {sum(r[2] for r in rounds):.2f} ms  "
              f"gathered per rank {sum(r[5] for r in rounds) / 2**20:.1f} MiB", flush=True)
        # the planner's link term (engine.hip shard_round_costs): the bytes a rank receives (= what it
        # sends, by symmetry) over link_gbps x min(G - 1, 7) links, added to the device time
        bw = PARAMS.get("link_gbps", 76.0) or 76.0
        link_ms = sum(r[5] for r in rounds) / (bw * 1e6 * min(G - 1, 7))
        print(f"G={G} plan link_gbps={PARAMS.get('link_gbps', 76.0)}: modelled per-rank wall "
              f"{sum(r[2] for r in rounds) + link_ms:.2f} ms = device {sum(r[2] for r in rounds):.2f} + "
              f"link {link_ms:.2f} (at {bw:g} GB/s per link); kinds "
              f"{''.join('DSAXCRrQ'[r[1]] for r in rounds)}", flush=True)
