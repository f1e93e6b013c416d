"""CPU: FLOOD restates main.go:65-89 (+ dedupe :113) — infected set after t
rounds is the BFS ball of radius t, rounds to converge = eccentricity of the
origin, and every informed node forwards exactly once (message accounting)."""
from collections import deque

import numpy as np
import pytest

import oracle_py as op
from gossip_hip.maelstrom import grid_topology, line_topology, total_topology, tree_topology


def adj_of(topo, n):
    return [[int(v[1:]) for v in topo[f"n{i}"]] for i in range(n)]


def bfs(adj, src):
    d = [-1] * len(adj)
    d[src] = 0
    q = deque([src])
    while q:
        u = q.popleft()
        for v in adj[u]:
            if d[v] < 0:
                d[v] = d[u] + 1
                q.append(v)
    return d


TOPOS = [("grid", grid_topology, 25), ("grid", grid_topology, 5), ("grid", grid_topology, 100),
         ("line", line_topology, 17), ("total", total_topology, 9), ("tree2", tree_topology, 31),
         ("tree4", lambda n: tree_topology(n, 4), 50)]


@pytest.mark.parametrize("name,fn,n", TOPOS)
def test_bfs_ball_and_eccentricity(name, fn, n):
    adj = adj_of(fn(n), n)
    for origin in sorted({0, n // 2, n - 1}):
        d = bfs(adj, origin)
        e = op.OracleEngine(n, 1, "flood", 0)
        e.set_topology(adj)
        e.inject(origin, 0)
        res = e.step(1000)
        assert res.rounds == max(d)  # rounds to converge = ecc(origin)
        for t, st in enumerate(res.stats):
            assert st["full_nodes"] == sum(1 for x in d if 0 <= x <= t + 1)
        # every node forwards once, to deg - 1 neighbours (deg for the origin)
        total = sum(s["messages"] for s in res.stats)
        last = [v for v in range(n) if d[v] == max(d)]
        expect = sum(len(adj[v]) - (v != origin) for v in range(n) if v not in last)
        assert total == expect


def test_grid25_corner_is_8_rounds():
    adj = adj_of(grid_topology(25), 25)
    e = op.OracleEngine(25, 1, "flood", 0)
    e.set_topology(adj)
    e.inject(0, 0)
    assert e.step(100).rounds == 8


def test_total_topology_one_round():
    n = 12
    e = op.OracleEngine(n, 1, "flood", 0)
    e.set_topology(adj_of(total_topology(n), n))
    e.inject(5, 0)
    res = e.step(10)
    assert res.rounds == 1 and res.stats[0]["messages"] == n - 1


def test_dedupe_reinject_is_noop():
    adj = adj_of(grid_topology(9), 9)
    e = op.OracleEngine(9, 2, "flood", 0, flags=1)
    e.set_topology(adj)
    e.inject(0, 0)
    e.inject(0, 0)  # duplicate client broadcast (main.go:113)
    h0 = e.state_hash()
    e2 = op.OracleEngine(9, 2, "flood", 0, flags=1)
    e2.set_topology(adj)
    e2.inject(0, 0)
    assert e2.state_hash() == h0
    assert e.step(50).stats == e2.step(50).stats


def test_disconnected_quiesces():
    adj = [[1], [0], [3], [2]]
    e = op.OracleEngine(4, 1, "flood", 0)
    e.set_topology(adj)
    e.inject(0, 0)
    res = e.step(100)
    assert res.stats[-1]["messages"] == 0 and not res.converged
    assert e.read(1) == [0] and e.read(2) == []


def test_monotone_random_modes():
    for mode in ("push", "pull", "pushpull"):
        e = op.OracleEngine(5000, 64, mode, 2, 3)
        e.inject_random()
        res = e.step(200)
        inf = res.infected.astype(np.int64)
        assert (np.diff(inf, axis=0) >= 0).all()
        assert res.converged and (inf[-1] == 5000).all()
