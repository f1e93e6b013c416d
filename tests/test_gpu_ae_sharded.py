"""GPU: sharded anti-entropy (SURVEY.md §8(e) Design B, row f4).

G HIP shard engines driven in lockstep through the gossip_ae_* protocol (stale-bit
all-gather, request / reply all-to-all, max-merge on the owner, the global max vector by a
MAX reduction) on one device — device copies stand in for RCCL, which the multi-GPU driver
(gossip_hip.sharded) uses — must equal the single-engine run and the oracle bit for bit:
per-round alive / full / messages / hash / per-component counts, and every row.
Reference: (*NodeState).Gossip, main.go:65-89 (each exchange = one request/reply)."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_py as op
from gossip_hip import Engine
from gossip_hip.engine import StepResult, churn_threshold as ct
from gossip_hip.sharded import lockstep_run

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)

CASES = [  # N, K, fanout, seed, fail, recover, G
    (1 << 16, 16, 1, 0x5EED0005, 0.01, 0.1, 4),
    (50_001, 5, 2, 0x5EED000A, 0.05, 0.3, 3),
    (4099, 64, 3, 3, 0.02, 0.2, 2),
    (777, 1, 1, 11, 0.0, 0.0, 2),
    (100, 8, 1, 5, 0.05, 0.3, 4),  # 64-node row blocks: shards of 64, 36, 0 and 0 nodes
]


def _run_single(cls, N, K, k, seed, fail, rec, **kw):
    e = cls(N, K, "antientropy", k, seed, flags=1, churn_fail=ct(fail), churn_recover=ct(rec), **kw)
    e.inject_random()
    a = e.step(5)
    e.inject(N // 2, K - 1)
    e.inject(3, 0)
    b = e.step(400)
    return a.stats + b.stats, e.read_rows(), e


@pytest.mark.parametrize("case", CASES, ids=[f"N{c[0]}-K{c[1]}-k{c[2]}-G{c[6]}" for c in CASES])
def test_ae_lockstep_equals_single_engine_and_oracle(case):
    N, K, k, seed, fail, rec, G = case
    want, rows, ref = _run_single(Engine, N, K, k, seed, fail, rec)
    ref.close()
    ostats, orows, _ = _run_single(op.OracleEngine, N, K, k, seed, fail, rec, threads=THREADS)
    assert ostats == want and np.array_equal(orows, rows)
    engines = [Engine(N, K, "antientropy", k, seed, flags=1, shard_rank=r, shard_count=G, churn_fail=ct(fail),
                      churn_recover=ct(rec)) for r in range(G)]
    for e in engines:
        e.inject_random()
    a, kinds = lockstep_run(engines, 5)
    for e in engines:
        e.inject(N // 2, K - 1)
        e.inject(3, 0)
    b, _ = lockstep_run(engines, 400)
    assert set(kinds) == {2}
    assert a + b == want
    for e in engines:
        assert np.array_equal(e.read_rows(), rows[e.lo:e.hi])
        e.close()


CFG5 = (1 << 26, 16, 1, 0x5EED0005, 0.01, 0.1)  # configs[4]: N, K, fanout, seed, fail, recover
CFG5_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cfg5_oracle.json")


def _digest_update(h, rows):
    h.update(memoryview(np.ascontiguousarray(rows, dtype="<u4")).cast("B"))


def _oracle_live(request):
    """The OpenMP oracle run itself (oracle/gossip_oracle.c ae_round, the restatement of main.go:65-89
    with each exchange one request/reply), in the golden file's format."""
    N, K, k, seed, fail, rec = CFG5
    o = op.OracleEngine(N, K, "antientropy", k, seed, flags=1, churn_fail=ct(fail), churn_recover=ct(rec),
                        threads=THREADS)
    o.inject_random()
    capman = request.config.pluginmanager.getplugin("capturemanager")
    stats, inf = [], []
    while len(stats) < 400:  # in slices, with a progress line: the oracle takes minutes at this size
        r = o.step(10)
        stats += r.stats
        inf += [[int(x) for x in row] for row in r.infected]
        with capman.global_and_fixture_disabled():  # a progress line past pytest's capture
            print(f"cfg5 oracle: {len(stats)} rounds", flush=True)
        if r.converged:
            break
    rows = o.read_rows()
    o.close()
    h = hashlib.sha256()
    _digest_update(h, rows)
    return {"rounds": len(stats), "stats": stats, "infected": inf, "rows_sha256": h.hexdigest(),
            "sample_rows": {}}


@pytest.fixture(scope="module")
def cfg5_oracle(request):
    """configs[4] at full size on the OpenMP oracle, to convergence: per-round stats (alive, full,
    messages, hash), per-component counts, and the SHA-256 of every row.  From
    tests/golden/cfg5_oracle.json (written by tests/golden/make_cfg5_golden.py from the same oracle;
    the live run costs ~200 s on the GPU box), or live with GOSSIP_CFG5_LIVE=1."""
    if os.environ.get("GOSSIP_CFG5_LIVE") == "1" or not os.path.exists(CFG5_GOLDEN):
        return _oracle_live(request)
    with open(CFG5_GOLDEN) as f:
        g = json.load(f)
    N, K, k, seed, fail, rec = CFG5
    assert g["config"]["N"] == N and g["config"]["K"] == K and int(g["config"]["seed"], 16) == seed
    return g


def _check_rows(want, parts):
    h = hashlib.sha256()
    for lo, rows in parts:
        _digest_update(h, rows)
        for n, v in want["sample_rows"].items():
            if lo <= int(n) < lo + len(rows):
                assert list(rows[int(n) - lo]) == v, n
    assert h.hexdigest() == want["rows_sha256"]


def test_cfg5_64M_single_engine_equals_oracle(cfg5_oracle):
    """configs[4] at full size (2^26 nodes, K = 16, fanout 1, churn 1 % / 10 %) on one HIP engine
    (dense rounds, then sparse rounds as planned) against the oracle."""
    want = cfg5_oracle
    N, K, k, seed, fail, rec = CFG5
    e = Engine(N, K, "antientropy", k, seed, flags=1, churn_fail=ct(fail), churn_recover=ct(rec))
    e.inject_random()
    got = e.step(400)
    assert got.rounds == want["rounds"] and got.converged
    assert got.stats == want["stats"]
    assert np.array_equal(got.infected, np.array(want["infected"], dtype=np.uint64))
    _check_rows(want, [(0, e.read_rows())])
    e.close()


def test_cfg5_64M_G8_lockstep_equals_oracle(cfg5_oracle):
    """configs[4] at full size as 8 shards of 2^23 rows (the sharded ANTIENTROPY protocol, DESIGN.md
    §5.3) against the oracle, to convergence."""
    want = cfg5_oracle
    N, K, k, seed, fail, rec = CFG5
    G = 8
    engines = [Engine(N, K, "antientropy", k, seed, flags=1, shard_rank=r, shard_count=G, churn_fail=ct(fail),
                      churn_recover=ct(rec)) for r in range(G)]
    for e in engines:
        e.inject_random()
    got, _ = lockstep_run(engines, 400)
    assert got == want["stats"]
    parts = []
    for e in engines:
        assert e.hi - e.lo == 1 << 23
        parts.append((e.lo, e.read_rows()))
        e.close()
    _check_rows(want, parts)
