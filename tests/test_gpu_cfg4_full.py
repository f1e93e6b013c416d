"""GPU, configs[3] at full size: 2^27 nodes, push-pull fanout 2, 64 rumors at their Philox
origins, seed 0x5EED0004 — the north star's 128M-node sweep.

Three results must agree bit for bit, round by round (stats, per-rumor counts) and in the
final state:
  * G = 8 shard engines of 2^24 nodes each, driven in lockstep through the sharded round
    protocol on one device (device copies stand in for the RCCL collectives; the 8-GPU
    node runs the same engine calls over RCCL: gossip_hip.sharded), for the auto, sparse,
    dense (state all-gather) and exchange round plans;
  * one engine holding all 2^27 nodes (the binned path past 4096 tiles, binned.hip V = 3);
  * the OpenMP oracle (oracle/gossip_oracle.c) at 2^27.
Reference: (*NodeState).Gossip, main.go:65-89, restated as rounds."""
import os

import numpy as np
import pytest

import oracle_py as op
from gossip_hip import Engine
from gossip_hip.sharded import lockstep_run

pytestmark = pytest.mark.gpu

N, R, K, SEED, G = 1 << 27, 64, 2, 0x5EED0004, 8
THREADS = min(16, os.cpu_count() or 1)
# auto: sparse rounds and exchange dense rounds (G = 8 >= xd_shards); dense: every round on the
# state all-gather; exchange: every round an exchange dense round; classcoded:
# every round on the class-coded all-gather (§5.1); auto_image: sparse rounds and dense rounds
# on the image, class-coded while few nodes are mixed
PLANS = {"auto": {}, "sparse": {"sparse_frac": 1.0}, "dense": {"sparse_frac": -1, "xd_shards": 0, "cc_frac": 0},
         "exchange": {"sparse_frac": -1}, "classcoded": {"sparse_frac": -1, "xd_shards": 0, "cc_frac": 1},
         "auto_image": {"xd_shards": 0}}


@pytest.fixture(scope="module")
def single_engine_run():
    e = Engine(N, R, "pushpull", K, SEED, flags=1)
    e.inject_random()
    res = e.step(64)
    full = e.read_shard()
    e.close()
    return res, full


def test_cfg4_single_engine_equals_oracle(single_engine_run):
    res, full = single_engine_run
    o = op.OracleEngine(N, R, "pushpull", K, SEED, flags=1, threads=THREADS)
    o.inject_random()
    ro = o.step(64)
    assert res.converged and res.stats == ro.stats
    assert np.array_equal(res.infected, ro.infected)
    assert np.array_equal(full, o.read_shard())
    o.close()


def test_cfg4_single_engine_equals_fixture(single_engine_run):
    """The same run against the committed oracle fixture (tests/golden/cfg4_oracle.json, the file
    bench.py checks every configs[3] line against): stats, per-rumor counts, final state digest."""
    import hashlib
    import json
    res, full = single_engine_run
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cfg4_oracle.json")) as f:
        fx = json.load(f)
    assert res.stats == fx["stats"]
    assert res.infected.tolist() == fx["infected"]
    words = np.ascontiguousarray(full[0], dtype="<u8")
    assert hashlib.sha256(memoryview(words).cast("B")).hexdigest() == fx["state_sha256"]


# one engine on other round paths against the same fixture: every round dense; every round sparse
ONE_PATHS = {"dense": {"sparse_frac": -1}, "sparse": {"sparse_frac": 1.0}}


@pytest.mark.parametrize("path", list(ONE_PATHS))
def test_cfg4_round_paths_equal_fixture(path):
    import hashlib
    import json
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cfg4_oracle.json")) as f:
        fx = json.load(f)
    e = Engine(N, R, "pushpull", K, SEED, flags=1, params=ONE_PATHS[path])
    e.inject_random()
    res = e.step(64)
    assert res.stats == fx["stats"]
    assert res.infected.tolist() == fx["infected"]
    words = np.ascontiguousarray(e.read_shard()[0], dtype="<u8")
    assert hashlib.sha256(memoryview(words).cast("B")).hexdigest() == fx["state_sha256"]
    e.close()


@pytest.mark.parametrize("plan", list(PLANS))
def test_cfg4_G8_lockstep_equals_single_engine(single_engine_run, plan):
    res, full = single_engine_run
    engines = [Engine(N, R, "pushpull", K, SEED, flags=1, shard_rank=r, shard_count=G, params=PLANS[plan])
               for r in range(G)]
    for e in engines:
        e.inject_random()
    got, kinds = lockstep_run(engines, 64)
    assert got == res.stats
    if plan == "sparse":
        assert set(kinds) == {1}
    elif plan == "dense":
        assert set(kinds) == {0}
    elif plan == "exchange":
        assert set(kinds) == {3}
    elif plan == "classcoded":
        assert set(kinds) == {4}
    for e in engines:
        assert e.hi - e.lo == 1 << 24
        assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])
        e.close()
