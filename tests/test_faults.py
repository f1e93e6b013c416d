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


def test_faults_rejected_for_flood():
    with pytest.raises(Exception):
        op.OracleEngine(25, 1, "flood", 0, 0, edge_loss=1)


def test_loss_threshold():
    assert loss_threshold(0.0) == 0 and loss_threshold(1.0) == 2**32 - 1 and loss_threshold(0.5) == 2**31
