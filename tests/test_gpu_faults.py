"""GPU: the fault model is the same on every round path and
equals the oracle bit for bit — per-round stats, per-rumor counts, final state —
with edge loss, partitions and both, including fanout > 4 (the per-edge draw
paths), sharded lockstep runs and healing a partition between steps."""
import numpy as np
import pytest

import oracle_py as op
from gossip_hip import FLAG_DENSE, FLAG_DIRECT, Engine, loss_threshold
from gossip_hip.sharded import lockstep_run

pytestmark = pytest.mark.gpu

CASES = [  # mode, k, R, N, seed, edge_loss, partitions
    ("pushpull", 2, 64, 3000, 0x5EED0003, loss_threshold(0.3), 0),
    ("push", 3, 1, 2001, 7, loss_threshold(0.1), 3),
    ("pull", 2, 5, 4096, 11, loss_threshold(0.2), 2),
    ("pushpull", 6, 7, 1500, 3, loss_threshold(0.25), 2),
]
IDS = ["pushpull-loss", "push-loss-parts", "pull-loss-parts", "pushpull-k6"]
PATHS = {"auto": (0, {}), "dense": (FLAG_DENSE, {}), "dense_filter": (0, {"sparse_frac": -1, "filter_frac": 0}),
         "sparse": (0, {"sparse_frac": 1.0, "alld_frac": 1e30}),
         "sparse_alld": (0, {"sparse_frac": 1.0, "alld_frac": 0}), "direct": (FLAG_DIRECT, {})}


def _oracle(case, rounds=200):
    mode, k, R, N, seed, loss, parts = case
    ref = op.OracleEngine(N, R, mode, k, seed, flags=1, edge_loss=loss, partitions=parts)
    ref.inject_random()
    return ref.step(rounds), ref.read_shard()


@pytest.mark.parametrize("path", list(PATHS))
@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_faults_every_path_equals_oracle(case, path):
    mode, k, R, N, seed, loss, parts = case
    want, full = _oracle(case)
    flags, params = PATHS[path]
    e = Engine(N, R, mode, k, seed, flags=1 | flags, edge_loss=loss, partitions=parts, params=params)
    e.inject_random()
    got = e.step(200)
    assert got.stats == want.stats
    assert np.array_equal(got.infected, want.infected)
    assert np.array_equal(e.read_shard(), full)
    e.close()


@pytest.mark.parametrize("plan", ["auto", "sparse", "dense"])
def test_faults_sharded_lockstep(plan):
    case = ("pushpull", 2, 64, 30011, 0x5EED0004, loss_threshold(0.25), 3)
    mode, k, R, N, seed, loss, parts = case
    want, full = _oracle(case)
    params = {} if plan == "auto" else {"sparse_frac": 1.0 if plan == "sparse" else -1}
    engines = [Engine(N, R, mode, k, seed, flags=1, shard_rank=r, shard_count=3, edge_loss=loss, partitions=parts,
                      params=params) for r in range(3)]
    for e in engines:
        e.inject_random()
    got, _ = lockstep_run(engines, 200)
    assert got == want.stats
    for e in engines:
        assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])
        e.close()


def test_heal_partition_gpu():
    N = 5000
    ref = op.OracleEngine(N, 3, "pushpull", 2, 1, flags=1, partitions=4)
    e = Engine(N, 3, "pushpull", 2, 1, flags=1, partitions=4)
    for x in (ref, e):
        x.inject(0, 0); x.inject(N - 1, 1); x.inject(N // 2, 2)
    a, b = ref.step(40), e.step(40)
    assert a.stats == b.stats and not b.converged
    for x in (ref, e):
        x.set_faults(loss_threshold(0.1), 0)
    a, b = ref.step(100), e.step(100)
    assert a.stats == b.stats and b.converged
    assert np.array_equal(ref.read_shard(), e.read_shard())
