"""GPU: multi-GPU rounds driven by the library itself (include/gossip.h
gossip_group_* / gossip_comm_init_rank).  G shard engines in one process, every round run by
the C++ driver (plan, collectives, kernels; the same protocol gossip_hip.sharded runs over
torch.distributed), equal one engine bit for bit — per-round stats, per-rumor counts and the
final state — for every plan kind: sparse rounds, the state all-gather, its class-coded form,
exchange rounds and sharded ANTIENTROPY.  On a one-GPU box the collectives are device copies
(transport 2); on distinct devices the same calls go over RCCL (transport 1).
Reference: (*NodeState).Gossip, main.go:65-89, driven from the caller's thread (main.go:118)."""
import numpy as np
import pytest

from gossip_hip import Engine, Group
from gossip_hip.engine import churn_threshold as ct, loss_threshold

pytestmark = pytest.mark.gpu

PLANS = {"auto": {}, "sparse": {"sparse_frac": 1.0}, "dense": {"sparse_frac": -1, "xd_shards": 0, "cc_frac": 0},
         "classcoded": {"sparse_frac": -1, "xd_shards": 0, "cc_frac": 1},
         "exchange": {"sparse_frac": -1, "xd_shards": 2}, "auto_exchange": {"xd_shards": 2},
         "replicated": {"sparse_frac": -1, "replicate": 1}, "auto_replicated": {"replicate": 1}}
CASES = [("pushpull", 2, 64, 1 << 20, 0x5EED0004, 4), ("push", 3, 1, 300001, 7, 3),
         ("pull", 1, 5, 100000, 11, 2), ("pushpull", 2, 5, 12, 3, 5)]
IDS = ["pushpull-1M-G4", "push-ragged-G3", "pull-G2", "pushpull-N12-G5-empty"]


def _one_engine(mode, k, R, N, seed, **kw):
    ref = Engine(N, R, mode, k, seed, flags=1, **kw)
    ref.inject_random()
    want = ref.step(300)
    full = ref.read_shard() if mode != "antientropy" else ref.read_rows()
    ref.close()
    return want, full


@pytest.mark.parametrize("plan", list(PLANS))
@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_group_equals_one_engine(case, plan):
    mode, k, R, N, seed, G = case
    want, full = _one_engine(mode, k, R, N, seed)
    with Group(N, R, mode, k, seed, flags=1, n_shards=G, devices=[0] * G, params=PLANS[plan]) as g:
        assert g.transport == 2  # one device: device copies
        g.inject_random()
        got = g.step(300)
        assert got.stats == want.stats
        assert np.array_equal(got.infected, want.infected)
        for e in g.shards:
            assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])


def test_group_faults_and_stall():
    N, R, k, seed, G = 30011, 64, 2, 0x5EED0004, 3
    kw = dict(edge_loss=loss_threshold(0.1), partitions=3, stall_rounds=3)
    want, full = _one_engine("pushpull", k, R, N, seed, **kw)
    with Group(N, R, "pushpull", k, seed, flags=1, n_shards=G, devices=[0] * G, **kw) as g:
        g.inject_random()
        got = g.step(300)
        assert got.stats == want.stats
        for e in g.shards:
            assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])


@pytest.mark.parametrize("G", [2, 4])
def test_group_antientropy(G):
    N, K, k, seed = 1 << 16, 16, 1, 0x5EED0005
    kw = dict(churn_fail=ct(0.01), churn_recover=ct(0.1))
    want, rows = _one_engine("antientropy", k, K, N, seed, **kw)
    with Group(N, K, "antientropy", k, seed, flags=1, n_shards=G, devices=[0] * G, **kw) as g:
        g.inject_random()
        got = g.step(400)
        assert got.stats == want.stats
        assert np.array_equal(got.infected, want.infected)
        for e in g.shards:
            assert np.array_equal(e.read_rows(), rows[e.lo:e.hi])


def test_group_steps_again_after_inject():
    """Rounds after a client broadcast mid-run: the group replans from the shards' own totals."""
    N, R, G = 200003, 3, 3
    ref = Engine(N, R, "pushpull", 2, 9, flags=1)
    with Group(N, R, "pushpull", 2, 9, flags=1, n_shards=G, devices=[0] * G) as g:
        for x in (ref, g):
            x.inject(5, 0)
            x.inject(N - 1, 1)
        a, b = ref.step(4), g.step(4)
        assert a.stats == b.stats
        for x in (ref, g):
            x.inject(77, 2)
        a, b = ref.step(100), g.step(100)
        assert a.stats == b.stats and b.converged
        full = ref.read_shard()
        for e in g.shards:
            assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])
    ref.close()


@pytest.fixture(scope="module")
def cfg4_one_engine():
    return _one_engine("pushpull", 2, 64, 1 << 27, 0x5EED0004)


@pytest.mark.parametrize("G", [2, 4, 8])
def test_cfg4_group_equals_one_engine(cfg4_one_engine, G):
    """configs[3] at full size, 2^27 nodes over G shards (bench.py's strong-scaling sweep: state
    all-gather rounds below 6 shards, exchange rounds at 8), every round run by the library."""
    N, R, k, seed = 1 << 27, 64, 2, 0x5EED0004
    want, full = cfg4_one_engine
    with Group(N, R, "pushpull", k, seed, flags=1, n_shards=G, devices=[0] * G) as g:
        g.inject_random()
        got = g.step(64)
        assert got.converged and got.stats == want.stats
        for e in g.shards:
            assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])


def _rccl_devices(G):
    import torch
    if torch.cuda.device_count() < G:
        pytest.skip(f"RCCL needs one device per shard: {G} shards, {torch.cuda.device_count()} device(s)")
    return list(range(G))


RCCL_PLANS = ["auto", "sparse", "classcoded", "exchange"]


@pytest.mark.parametrize("dev", [0, 1])
@pytest.mark.parametrize("plan", RCCL_PLANS)
@pytest.mark.parametrize("G", [2, 4, 8])
def test_rccl_group_equals_one_engine(plan, G, dev):
    """The RCCL transport (transport 1: ncclCommInitAll over distinct devices, collectives on the
    engines' streams, the side-stream all-gather, grouped ncclSend / ncclRecv all-to-alls) against
    one engine: every plan kind, per-round stats, per-rumor counts, final state.  dev 1 turns on
    the opt-in device-value collectives (param rccl_dev_collectives; off by default)."""
    devs = _rccl_devices(G)
    mode, k, R, N, seed = "pushpull", 2, 64, (1 << 20) + 77, 0x5EED0004
    want, full = _one_engine(mode, k, R, N, seed)
    params = dict(PLANS[plan], **({"xd_shards": 2} if plan in ("exchange", "auto") else {}))
    params["rccl_dev_collectives"] = dev
    with Group(N, R, mode, k, seed, flags=1, n_shards=G, devices=devs, transport=1, params=params) as g:
        assert g.transport == 1
        g.inject_random()
        got = g.step(300)
        assert got.stats == want.stats
        assert np.array_equal(got.infected, want.infected)
        for e in g.shards:
            assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])


@pytest.mark.parametrize("G", [2, 4])
def test_rccl_group_antientropy(G):
    devs = _rccl_devices(G)
    N, K, k, seed = 1 << 16, 16, 1, 0x5EED0005
    kw = dict(churn_fail=ct(0.01), churn_recover=ct(0.1))
    want, rows = _one_engine("antientropy", k, K, N, seed, **kw)
    with Group(N, K, "antientropy", k, seed, flags=1, n_shards=G, devices=devs, transport=1, **kw) as g:
        assert g.transport == 1
        g.inject_random()
        got = g.step(400)
        assert got.stats == want.stats
        for e in g.shards:
            assert np.array_equal(e.read_rows(), rows[e.lo:e.hi])


def test_rccl_group_rejects_shared_device():
    from gossip_hip import GossipError
    with pytest.raises(GossipError):
        Group(1000, 1, "push", 1, 1, n_shards=2, devices=[0, 0], transport=1)


def test_step_without_collectives_fails_loudly():
    from gossip_hip import GossipError
    e = Engine(1000, 1, "push", 1, 1, shard_rank=0, shard_count=2)
    e.inject(0, 0)
    with pytest.raises(GossipError):
        e.step(5)
    e.close()
