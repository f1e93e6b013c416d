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
    """N Maelstrom nodes in one or more engines, FLOOD mode (reference-faithful).

    The reference's MessageKeeper holds any number of values (main.go:35-39).  Each
    engine holds `page_values` rumor slots; the values fill pages in arrival order and a
    full page opens the next engine.  FLOOD rounds are independent per value bit, so a
    value's flood in its page is exactly its flood in one big engine.

    Broadcasts before any `topology`: the reference gossips them over a nil topology
    (main.go:72 ranges over no neighbours) and never forwards them later; here the page
    runs one round over an empty topology, which marks them forwarded (S_{t-1} = S_t).
    """

    def __init__(self, n_nodes: int, max_values: int = 0, engine_factory=None, page_values: int = 1024):
        self._factory = engine_factory or (lambda **kw: Engine(**kw))
        self.n = n_nodes
        self.max_values = max_values          # 0 = no limit
        self.page_values = max(1, min(page_values, 4096) if not max_values else min(page_values, max_values, 4096))
        self.ids = [node_id(i) for i in range(n_nodes)]
        self.index = {s: i for i, s in enumerate(self.ids)}
        self.slot_of = {}    # value -> global slot   (≙ MessageKeeper.broadcasted, main.go:24)
        self.values = []     # global slot -> value   (≙ MessageKeeper.messages, main.go:23)
        self.pages = []      # engines; slot s lives in pages[s // page_values], bit s % page_values
        self.adj = [[] for _ in range(n_nodes)]
        self.has_topology = False
        self._dirty = set()  # pages with values injected since their last gossip
        self._new_page()

    @property
    def engine(self):
        """The first page (single-page clusters: the engine)."""
        return self.pages[0]

    def _new_page(self):
        e = self._factory(n_nodes=self.n, n_rumors=self.page_values, mode="flood", fanout=0, seed=0)
        e.set_topology(self.adj)  # empty until the topology message arrives
        self.pages.append(e)
        return e

    def topology(self, topo: dict) -> None:
        """`topology` handler (main.go:132-149): replaces the neighbour map wholesale."""
        adj = [[] for _ in range(self.n)]
        for src, nbrs in topo.items():
            adj[self.index[src]] = [self.index[v] for v in nbrs]
        self.adj = adj
        for e in self.pages:
            e.set_topology(adj)
        self.has_topology = True

    def broadcast(self, node: str, message: int) -> None:
        """Client `broadcast` of `message` to `node` (main.go:102-121)."""
        slot = self.slot_of.get(message)
        if slot is None:
            if self.max_values and len(self.values) >= self.max_values:
                raise ValueError(f"more than {self.max_values} distinct values")
            slot = len(self.values)
            self.slot_of[message] = slot
            self.values.append(message)
            if slot // self.page_values >= len(self.pages):
                self._new_page()
        p = slot // self.page_values
        self.pages[p].inject(self.index[node], slot % self.page_values)
        self._dirty.add(p)

    def gossip(self, max_rounds: int = 1 << 16):
        """Runs flood rounds until every node holds every value or nothing is in flight
        (every page that received a broadcast since its last gossip).  Returns the
        result of the last page stepped; `messages` of all pages are summed per round."""
        res = None
        for p in sorted(self._dirty):
            r = self.pages[p].step(max_rounds if self.has_topology else 1)
            if res is None:
                res = r
            else:  # merge: rounds = the longest flood, messages added per round
                for i, st in enumerate(r.stats):
                    if i < len(res.stats):
                        res.stats[i]["messages"] += st["messages"]
                    else:
                        res.stats.append(dict(st))
                res.rounds = max(res.rounds, r.rounds)
        self._dirty.clear()
        if res is None:
            res = self.pages[0].step(0)
        return res

    def read(self, node: str) -> list:
        """`read` handler (main.go:123-130)."""
        out = []
        for p, e in enumerate(self.pages):
            base = p * self.page_values
            out.extend(self.values[base + s] for s in e.read(self.index[node]) if base + s < len(self.values))
        return out
