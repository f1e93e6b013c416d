"""Maelstrom-shaped façade over the engine (the reference's handler set).

The reference is one Maelstrom "broadcast" node process (main.go:99-158) whose
handlers are `topology` (:132-149), `broadcast` (:102-121) and `read`
(:123-130).  `Cluster` exposes the same three operations for a whole cluster of
nodes held in one engine, with Maelstrom node ids ("n0", "n1", ...), int64
message values, and the FLOOD mode that restates Gossip (:65-89) as rounds.

Values are mapped to rumor slots in arrival order, as MessageKeeper keeps
them in arrival order (Append, main.go:35-39); reads return the values a node
holds as a set sorted by slot (the reference's duplicate-on-race behaviour,
SURVEY.md §5, is not reproduced).
"""
from __future__ import annotations

import math

from .engine import Engine


def node_id(i: int) -> str:
    return f"n{i}"


def grid_topology(n: int) -> dict:
    """Maelstrom-style grid: row-major on a ceil(sqrt(n))-wide grid, 4-neighbourhood."""
    w = max(1, math.isqrt(n - 1) + 1) if n > 1 else 1
    topo = {}
    for i in range(n):
        r, c = divmod(i, w)
        nb = []
        for rr, cc in ((r - 1, c), (r + 1, c), (r, c - 1), (r, c + 1)):
            if 0 <= cc < w and rr >= 0:
                j = rr * w + cc
                if j < n:
                    nb.append(j)
        topo[node_id(i)] = [node_id(j) for j in nb]
    return topo


def line_topology(n: int) -> dict:
    return {node_id(i): [node_id(j) for j in (i - 1, i + 1) if 0 <= j < n] for i in range(n)}


def total_topology(n: int) -> dict:
    return {node_id(i): [node_id(j) for j in range(n) if j != i] for i in range(n)}


def tree_topology(n: int, branching: int = 2) -> dict:
    topo = {node_id(i): [] for i in range(n)}
    for i in range(1, n):
        p = (i - 1) // branching
        topo[node_id(i)].append(node_id(p))
        topo[node_id(p)].append(node_id(i))
    return topo


class Cluster:
    """N Maelstrom nodes in one engine, FLOOD mode (reference-faithful)."""

    def __init__(self, n_nodes: int, max_values: int = 64, engine_factory=None):
        factory = engine_factory or (lambda **kw: Engine(**kw))
        self.engine = factory(n_nodes=n_nodes, n_rumors=max_values, mode="flood", fanout=0, seed=0)
        self.n = n_nodes
        self.ids = [node_id(i) for i in range(n_nodes)]
        self.index = {s: i for i, s in enumerate(self.ids)}
        self.slot_of = {}    # value -> slot   (≙ MessageKeeper.broadcasted, main.go:24)
        self.values = []     # slot -> value   (≙ MessageKeeper.messages, main.go:23)
        self.has_topology = False

    def topology(self, topo: dict) -> None:
        """`topology` handler (main.go:132-149): replaces the neighbour map wholesale."""
        adj = [[] for _ in range(self.n)]
        for src, nbrs in topo.items():
            adj[self.index[src]] = [self.index[v] for v in nbrs]
        self.engine.set_topology(adj)
        self.has_topology = True

    def broadcast(self, node: str, message: int) -> None:
        """Client `broadcast` of `message` to `node` (main.go:102-121)."""
        slot = self.slot_of.get(message)
        if slot is None:
            if len(self.values) >= self.engine.n_rumors:
                raise ValueError(f"more than {self.engine.n_rumors} distinct values")
            slot = len(self.values)
            self.slot_of[message] = slot
            self.values.append(message)
        self.engine.inject(self.index[node], slot)

    def gossip(self, max_rounds: int = 1 << 16):
        """Runs flood rounds until every node holds every value or nothing is in flight."""
        return self.engine.step(max_rounds)

    def read(self, node: str) -> list:
        """`read` handler (main.go:123-130)."""
        return [self.values[s] for s in self.engine.read(self.index[node]) if s < len(self.values)]
