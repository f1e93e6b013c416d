"""numpy_ref.py — TEST INFRASTRUCTURE ONLY.

An independent, vectorised numpy restatement of the round model,
written separately from the C oracle (oracle/gossip_oracle.c) so the two can be
cross-checked.  It generates the committed golden fixtures in tests/golden/
(tests/golden/make_golden.py).  Never imported by the product path.

Reference anchors (0xSherlokMo/gossip-protocol, main.go):
  flood      — (*NodeState).Gossip main.go:65-89: once-only forward to
               Topology[self] (:72) minus the sender (:73-75); dedupe :113.
  inject     — broadcast handler main.go:102-117.
  readout    — read handler main.go:123-130.
Random modes, Philox peers, multi-rumor words and the state hash are
build-defined (SURVEY.md §8 round model), not present in the reference.
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
GOLD = 0x9E3779B97F4A7C15
MASK64 = (1 << 64) - 1


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 over arrays (Random123 / rocRAND philox4x32_10.h:270-302)."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint32) for c in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    c0, c1, c2, c3 = (c.copy() for c in (c0, c1, c2, c3))
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = c0.astype(np.uint64) * M0
            p1 = c2.astype(np.uint64) * M1
            n0 = (p1 >> np.uint64(32)).astype(np.uint32) ^ c1 ^ k0
            n1 = p1.astype(np.uint32)
            n2 = (p0 >> np.uint64(32)).astype(np.uint32) ^ c3 ^ k1
            n3 = p0.astype(np.uint32)
            c0, c1, c2, c3 = n0, n1, n2, n3
            k0 = np.uint32((int(k0) + int(W0)) & 0xFFFFFFFF)
            k1 = np.uint32((int(k1) + int(W1)) & 0xFFFFFFFF)
    return c0, c1, c2, c3


def peers(seed: int, n_nodes: int, t: int, k: int, nodes=None) -> np.ndarray:
    """p_j(n, t) for all n (rows) and j < k (cols); DESIGN.md §2.2."""
    n = np.arange(n_nodes, dtype=np.uint64) if nodes is None else np.asarray(nodes, dtype=np.uint64)
    out = np.empty((n.size, k), dtype=np.uint64)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for blk in range((k + 3) // 4):
        x = philox4x32_10(n.astype(np.uint32), np.uint32(t), np.uint32(0), np.uint32(blk), k0, k1)
        for q in range(4):
            j = blk * 4 + q
            if j >= k:
                break
            p = (x[q].astype(np.uint64) * np.uint64(n_nodes - 1)) >> np.uint64(32)
            p = p + (p >= n).astype(np.uint64)
            out[:, j] = p
    return out


def origins(seed: int, n_nodes: int, n_rumors: int) -> np.ndarray:
    """origin(r): Philox stream tag 2."""
    r = np.arange(n_rumors, dtype=np.uint32)
    x = philox4x32_10(r, 0, 2, 0, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    return ((x[0].astype(np.uint64) * np.uint64(n_nodes)) >> np.uint64(32)).astype(np.int64)


def mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = z ^ (z >> np.uint64(30))
        z = z * np.uint64(0xBF58476D1CE4E5B9)
        z = z ^ (z >> np.uint64(27))
        z = z * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def state_hash(S: np.ndarray) -> int:
    """Σ over nonzero words of mix64(word + (w*N+n)*GOLD) mod 2^64; S is [W, N]."""
    W, N = S.shape
    idx = np.arange(W * N, dtype=np.uint64).reshape(W, N)
    with np.errstate(over="ignore"):
        v = mix64(S + idx * np.uint64(GOLD))
    v = np.where(S != 0, v, np.uint64(0))
    return int(sum(int(x) for x in v.ravel().tolist()) & MASK64) if v.size < 4096 else \
        int(np.sum(v, dtype=np.uint64))


def full_masks(R: int) -> np.ndarray:
    W = (R + 63) // 64
    m = []
    for w in range(W):
        bits = R - 64 * w
        m.append((1 << 64) - 1 if bits >= 64 else (1 << bits) - 1)
    return np.array(m, dtype=np.uint64)


def stats_of(S: np.ndarray, R: int):
    W, N = S.shape
    fm = full_masks(R)
    full = int(np.all((S & fm[:, None]) == fm[:, None], axis=0).sum())
    bits = np.unpackbits(S.view(np.uint8).reshape(W, N, 8), axis=2, bitorder="little")  # [W,N,64]
    inf = bits.sum(axis=1, dtype=np.int64).reshape(W * 64)[:R]
    return full, [int(x) for x in inf]


def loss_draw(seed: int, nodes, t: int, j: int, value: int = 0) -> np.ndarray:
    """Philox({n, t, 4 | value << 16, j>>2})[j&3]: the loss draw of edge j of node n in round t
    (DESIGN.md §2.8); FLOOD walks draw one per message, value = the value's slot (§2.9)."""
    n = np.asarray(nodes, dtype=np.uint32)
    x = philox4x32_10(n, np.uint32(t), np.uint32(4 | (value << 16)), np.uint32(j >> 2), seed & 0xFFFFFFFF,
                      (seed >> 32) & 0xFFFFFFFF)
    return x[j & 3]


def edge_lost(seed, N, loss, parts, n, p, t, j, value: int = 0) -> np.ndarray:
    """The edge n -> p (slot j of n, round t) is lost: partition or loss draw (DESIGN.md §2.8;
    value: a FLOOD walk's message, one draw per value, §2.9)."""
    n = np.asarray(n, dtype=np.int64)
    p = np.asarray(p, dtype=np.int64)
    lost = np.zeros(n.shape, dtype=bool)
    if parts > 1:
        lost |= (n * parts) // N != (p * parts) // N
    if loss:
        lost |= loss_draw(seed, n, t, j, value) < np.uint32(loss)
    return lost


def popcount(x) -> int:
    return bin(int(x)).count("1")


class Sim:
    """Unsharded reference loop.  mode: 'flood' | 'push' | 'pull' | 'pushpull'.

    Faults (the reference's lossy SyncRPC with a 2 s context and
    unbounded retries, main.go:77-87): edge_loss / partitions lose edges; stall_rounds D
    restates the expired-context stall —
      random modes: a node whose initiated exchanges were lost (any of them) in D rounds in
        a row stops initiating exchanges (it still answers pulls and receives pushes);
      flood: one walk per (node, value) down the node's topology row in the topology
        message's order (duplicates kept), one blocking SyncRPC at a time: a lost attempt
        holds every later neighbour back until it is delivered (retried each round); after D
        lost attempts on one neighbour (D > 0) its context has expired and the walk never
        moves on — it keeps retrying that neighbour every round (each retry a message that
        delivers when not lost), the later neighbours never get the value from this node.
    """

    def __init__(self, n_nodes, n_rumors, mode, fanout=0, seed=0, topology=None, edge_loss=0, partitions=0,
                 stall_rounds=0):
        self.N, self.R, self.mode, self.k, self.seed = n_nodes, n_rumors, mode, fanout, seed
        self.loss, self.parts, self.D = edge_loss, partitions, stall_rounds
        self.W = (n_rumors + 63) // 64
        self.S = np.zeros((self.W, n_nodes), dtype=np.uint64)
        self.Sprev = np.zeros_like(self.S)
        self.t = 0
        self.streak = np.zeros(n_nodes, dtype=np.int64)  # random modes, stall_rounds > 0
        self.adj = None
        if topology is not None:
            # rows as sets
            self.adj = [sorted(set(int(v) for v in topology[u])) for u in range(n_nodes)]
            src, dst = [], []
            for u, row in enumerate(self.adj):
                for v in row:
                    src.append(u)
                    dst.append(v)
            self.src = np.array(src, dtype=np.int64)
            self.dst = np.array(dst, dtype=np.int64)
            self.deg = np.array([len(r) for r in self.adj], dtype=np.int64)
            self.skip = np.zeros_like(self.S)
            # flood with faults: per out-edge state (edge e = position in the CSR of sorted rows)
            self.edge_faults = bool(edge_loss or partitions > 1 or stall_rounds)
            E = len(self.src)
            self.row0 = np.concatenate([[0], np.cumsum(self.deg)]).astype(np.int64)
            # flood with faults: the walks, rows in the message's order
            self.rows = [[int(v) for v in topology[u]] for u in range(n_nodes)]
            self.cur = np.zeros((n_nodes, n_rumors), dtype=np.int64)   # next position in the row
            self.att = np.zeros((n_nodes, n_rumors), dtype=np.int64)   # lost attempts on that position
            self.snd = np.full((n_nodes, n_rumors), -1, dtype=np.int64)  # first sender (-1: a client)

    def inject(self, node, rumor):
        if self.adj is not None and self.edge_faults and not self._has(self.S, node, rumor):
            self.cur[node, rumor], self.att[node, rumor], self.snd[node, rumor] = 0, 0, -1
        self.S[rumor // 64, node] |= np.uint64(1 << (rumor % 64))

    @staticmethod
    def _has(S, node, x):
        return (int(S[x // 64, node]) >> (x % 64)) & 1 == 1

    def inject_random(self):
        for r, o in enumerate(origins(self.seed, self.N, self.R)):
            self.inject(int(o), r)

    def _flood_faults_round(self, S, Sn):
        """FLOOD with faults (main.go:72-87): every walk of a value u held at the
        start of the round goes down u's row from its cursor.  Position c of u's row is lost in
        round t like a random-mode edge (partition, or Philox({u, t, 4 | x << 16, c >> 2})[c & 3] <
        edge_loss: one draw per message, each value being its own SyncRPC, main.go:81); the first
        sender is skipped without a message (:73)."""
        D = self.D
        msgs = 0
        first = {}  # (w, x) -> lowest u that delivered x to w (w did not hold x)
        for u in range(self.N):
            row = self.rows[u]
            for x in range(self.R):
                if not self._has(S, u, x):
                    continue
                c, a, s = int(self.cur[u, x]), int(self.att[u, x]), int(self.snd[u, x])
                while c < len(row):
                    w = row[c]
                    if w == s:  # main.go:73
                        c += 1
                        continue
                    msgs += 1
                    if bool(edge_lost(self.seed, self.N, self.loss, self.parts, [u], [w], self.t, c, x)[0]):
                        a += 1
                        break
                    if not self._has(S, w, x):
                        first[(w, x)] = min(first.get((w, x), u), u)
                        Sn[x // 64, w] |= np.uint64(1 << (x % 64))
                    if D and a >= D:  # expired context: delivered, but the walk never moves on
                        break
                    c, a = c + 1, 0
                self.cur[u, x], self.att[u, x] = c, a
        for (w, x), u in first.items():  # walks of the values learned this round start next round
            self.cur[w, x], self.att[w, x], self.snd[w, x] = 0, 0, u
        return msgs

    def round(self):
        S = self.S
        Sn = S.copy()
        msgs = 0
        if self.mode == "flood" and self.edge_faults:
            msgs = self._flood_faults_round(S, Sn)
            self.Sprev = S
        elif self.mode == "flood":
            F = S & ~self.Sprev
            for w in range(self.W):
                # messages sent this round: |F[v]|*deg(v) - skipped senders (main.go:72-75)
                pc = np.array([bin(int(x)).count("1") for x in F[w]], dtype=np.int64)
                pk = np.array([bin(int(x)).count("1") for x in (F[w] & self.skip[w])], dtype=np.int64)
                msgs += int((pc * self.deg).sum() - pk.sum())
                np.bitwise_or.at(Sn[w], self.dst, F[w][self.src])
                new = Sn[w] & ~S[w]
                # first (lowest-id) sender per (v, bit); skip if it is in Adj(v)
                sk = np.zeros(self.N, dtype=np.uint64)
                seen = np.zeros(self.N, dtype=np.uint64)
                order = np.lexsort((self.src, self.dst))  # by dst, then src ascending
                for e in order:
                    u, v = self.src[e], self.dst[e]
                    c = F[w][u] & new[v] & ~seen[v]
                    if c:
                        if u in self.adj[v]:
                            sk[v] |= c
                        seen[v] |= c
                self.skip[w] = sk
            self.Sprev = S
        else:
            P = peers(self.seed, self.N, self.t, self.k).astype(np.int64)
            n = np.arange(self.N, dtype=np.int64)
            lost = np.stack([edge_lost(self.seed, self.N, self.loss, self.parts, n, P[:, j], self.t, j)
                             for j in range(self.k)], axis=1)
            stalled = self.streak >= self.D if self.D else np.zeros(self.N, dtype=bool)
            live = ~lost & ~stalled[:, None]  # a stalled node initiates nothing
            for w in range(self.W):
                for j in range(self.k):
                    src = n[live[:, j]]
                    dst = P[live[:, j], j]
                    if self.mode in ("pull", "pushpull"):
                        np.bitwise_or.at(Sn[w], src, S[w][dst])
                    if self.mode in ("push", "pushpull"):
                        np.bitwise_or.at(Sn[w], dst, S[w][src])
            if self.D:
                lost_any = lost.any(axis=1)
                self.streak = np.where(stalled, self.streak, np.where(lost_any, self.streak + 1, 0))
        self.S = Sn
        full, inf = stats_of(Sn, self.R)
        st = dict(round=self.t, full=full, converged=int(full == self.N), messages=msgs,
                  hash=state_hash(Sn), infected=inf)
        self.t += 1
        return st

    def run(self, max_rounds):
        out = []
        for _ in range(max_rounds):
            st = self.round()
            out.append(st)
            if st["converged"] or (self.mode == "flood" and st["messages"] == 0):
                break
        return out


class AntiEntropySim:
    """Version-vector anti-entropy with churn, unsharded, vectorised.

    V[n, c] uint32; alive[n] bool.  Round t: churn by the word x = Philox({n, t, 0, 0})[3] for
    fanout k <= 3 (the first peer draw's spare word), else Philox({n, t, 1, 0})[0] (x < fail
    kills an alive node, x < recover revives a dead one), then over every edge
    (n, p_j(n, t)) with both ends alive, both ends take the elementwise max of
    the two S_t vectors.  Stats: alive count, alive nodes equal to the global
    max vector (constant between injections), per-component counts, hash.
    """

    def __init__(self, n_nodes, k_comp, fanout, seed, fail, recover):
        self.N, self.K, self.k, self.seed, self.fail, self.rec = n_nodes, k_comp, fanout, seed, fail, recover
        self.V = np.zeros((n_nodes, k_comp), dtype=np.uint32)
        self.alive = np.ones(n_nodes, dtype=bool)
        self.t = 0

    def inject_random(self):
        n = np.arange(self.N, dtype=np.uint32)
        k0, k1 = self.seed & 0xFFFFFFFF, (self.seed >> 32) & 0xFFFFFFFF
        for c0 in range(0, self.K, 4):
            x = philox4x32_10(n, np.uint32(c0 // 4), np.uint32(3), np.uint32(0), k0, k1)
            for q in range(4):
                if c0 + q < self.K:
                    self.V[:, c0 + q] = x[q] & np.uint32(0xFFFF)

    def inject(self, node, comp):
        self.V[node, comp] += np.uint32(1)

    def round(self):
        N = self.N
        k0, k1 = self.seed & 0xFFFFFFFF, (self.seed >> 32) & 0xFFFFFFFF
        n = np.arange(N, dtype=np.uint32)
        if self.k <= 3:
            x0 = philox4x32_10(n, np.uint32(self.t), np.uint32(0), np.uint32(0), k0, k1)[3]
        else:
            x0 = philox4x32_10(n, np.uint32(self.t), np.uint32(1), np.uint32(0), k0, k1)[0]
        alive = np.where(self.alive, ~(x0 < np.uint32(self.fail)), x0 < np.uint32(self.rec))
        P = peers(self.seed, N, self.t, self.k).astype(np.int64)
        V = self.V
        Vn = V.copy()
        msgs = 0
        for j in range(self.k):
            p = P[:, j]
            e = alive & alive[p]
            src = np.nonzero(e)[0]
            dst = p[e]
            msgs += int(src.size)
            np.maximum.at(Vn, src, V[dst])  # pull
            np.maximum.at(Vn, dst, V[src])  # push
        self.V, self.alive = Vn, alive
        target = V.max(axis=0) if N else V[0]
        eq = Vn == target[None, :]
        full = int((eq.all(axis=1) & alive).sum())
        inf = [int(x) for x in (eq & alive[:, None]).sum(axis=0)]
        idx = (np.arange(self.K, dtype=np.uint64)[None, :] * np.uint64(N) + np.arange(N, dtype=np.uint64)[:, None])
        with np.errstate(over="ignore"):
            h = mix64(Vn.astype(np.uint64) + idx * np.uint64(GOLD))
        h = int(np.sum(np.where(Vn != 0, h, np.uint64(0)), dtype=np.uint64))
        st = dict(round=self.t, full=full, alive=int(alive.sum()), converged=int(full == int(alive.sum())),
                  messages=msgs, hash=h, infected=inf)
        self.t += 1
        return st

    def run(self, max_rounds):
        out = []
        for _ in range(max_rounds):
            st = self.round()
            out.append(st)
            if st["converged"]:
                break
        return out
