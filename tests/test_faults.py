"""CPU: the fault model (SURVEY.md §8(f) 3 — the reference's
lossy SyncRPC, main.go:77-87) on the oracle: partitions confine rumors to their
block, healing a partition lets them through, loss only slows dissemination,
and the sharded protocol under faults equals the unsharded run (gloo).
Parity of the HIP paths against this oracle is tests/test_gpu_faults.py."""
import numpy as np
import pytest

import oracle_py as op
from gossip_hip import loss_threshold


def _run(e, rounds):
    res = e.step(rounds)
    return res, e.read_shard()[0]


def test_partition_confines_rumors():
    N, P = 4000, 2
    e = op.OracleEngine(N, 1, "pushpull", 2, 21, flags=1, partitions=P)
    e.inject(10, 0)  # block 0 = nodes [0, 2000)
    res, s = _run(e, 60)
    assert not res.converged
    assert (s[:N // 2] == 1).all() and (s[N // 2:] == 0).all()  # the whole block, nothing beyond it


def test_heal_partition():
    N = 3001
    e = op.OracleEngine(N, 1, "push", 3, 5, flags=1, partitions=3)
    e.inject(0, 0)
    res, s = _run(e, 80)
    assert not res.converged and s.sum() == (N + 2) // 3  # block 0 of 3 (ceil split)
    e.set_faults(0, 0)
    res, s = _run(e, 80)
    assert res.converged and (s == 1).all()


def test_loss_only_slows():
    rounds = []
    for p in (0.0, 0.3, 0.6):
        e = op.OracleEngine(2000, 8, "pushpull", 2, 9, flags=1, edge_loss=loss_threshold(p))
        e.inject_random()
        res, s = _run(e, 200)
        assert res.converged and (s == 0xFF).all()
        rounds.append(res.rounds)
    assert rounds[0] <= rounds[1] <= rounds[2] and rounds[0] < rounds[2]


def test_flood_faults_single_shard_only():
    """FLOOD retries keep per-edge state on one shard; a sharded FLOOD engine, or
    an ANTIENTROPY one (churn is its fault model), rejects faults."""
    op.OracleEngine(25, 1, "flood", 0, 0, edge_loss=1)
    with pytest.raises(Exception):
        op.OracleEngine(25, 1, "flood", 0, 0, edge_loss=1, shard_count=2)
    with pytest.raises(Exception):
        op.OracleEngine(25, 1, "antientropy", 1, 0, stall_rounds=2)
    e = op.OracleEngine(25, 1, "flood", 0, 0)  # created without faults: no per-edge state to retry from
    with pytest.raises(Exception):
        e.set_faults(1, 0)


def test_stall_mode_properties():
    """Stall mode: more stall-prone settings never spread further; without losses
    nothing ever stalls; a long partition stalls every node that keeps losing its exchanges."""
    N = 3000
    full = []
    for d in (0, 6, 3, 1):
        e = op.OracleEngine(N, 8, "pushpull", 2, 9, flags=1, edge_loss=loss_threshold(0.15), stall_rounds=d)
        e.inject_random()
        res = e.step(60)
        full.append(res.stats[-1]["full_nodes"])
    assert full[0] == N and full[0] >= full[1] >= full[2] >= full[3] and full[3] < N
    a = op.OracleEngine(N, 8, "pushpull", 2, 9, flags=1, stall_rounds=1)
    b = op.OracleEngine(N, 8, "pushpull", 2, 9, flags=1)
    for x in (a, b):
        x.inject_random()
    assert a.step(60).stats == b.step(60).stats


def test_loss_threshold():
    assert loss_threshold(0.0) == 0 and loss_threshold(1.0) == 2**32 - 1 and loss_threshold(0.5) == 2**31


def test_flood_new_topology_ends_walks():
    """a topology message ends every walk, so a value already held is not sent
    again over the new rows; a value injected after it starts a walk on them.  (main.go:72 reads
    the row once per goroutine, so in the reference an in-flight walk would finish on the old
    row: a documented divergence.)"""
    N = 6
    e = op.OracleEngine(N, 2, "flood", 0, 1, flags=1, stall_rounds=1)
    e.set_topology([[1], [], [], [], [], []])  # 0 -> 1 only
    e.inject(0, 0)
    e.step(10)
    assert e.read(1) == [0] and e.read(2) == []
    e.set_topology([[2, 3], [4], [], [], [], []])
    res = e.step(10)
    assert res.stats[-1]["messages"] == 0 and e.read(2) == [] and e.read(4) == []  # walks ended
    e.inject(0, 1)  # a new value walks the new rows: 0 -> 2, 3
    e.step(10)
    assert e.read(2) == [1] and e.read(3) == [1] and e.read(4) == []
    e.close()
