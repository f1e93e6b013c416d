"""GPU parity: the HIP engine (libgossip_hip.so, through the C ABI) against
the CPU oracle and the committed golden vectors — bit-exact per round."""
import os

import numpy as np
import pytest
import torch

import oracle_py as op
from conftest import inject_case
from gossip_hip import FLAG_DENSE, FLAG_DIRECT, FLAG_TIMING, Cluster, Engine, grid_topology
from gossip_hip.engine import GossipError

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)


def test_device_philox_kat(golden):
    e = Engine(16, 1, "push", 1, 0)
    ctr = np.array([v["ctr"] for v in golden["philox_kat"]], dtype=np.uint32)
    for i, v in enumerate(golden["philox_kat"]):
        out = e.philox_device(ctr[i:i + 1], v["key"])
        assert [int(x) for x in out[0]] == v["out"]
    # a bulk batch against the oracle
    rng = np.random.default_rng(1)
    c = rng.integers(0, 2**32, size=(4096, 4), dtype=np.uint64).astype(np.uint32)
    out = e.philox_device(c, [0x5EED0003, 0])
    for i in range(0, 4096, 257):
        assert [int(x) for x in out[i]] == op.philox([int(x) for x in c[i]], [0x5EED0003, 0])


# round paths of the random modes, all bit-identical:
#   auto   — default: sparse frontier rounds while one class dominates, dense binned rounds otherwise
#   dense  — every round on the binned LDS pipeline
#   sparse — every round on the frontier kernels (sparse_frac = 1 lifts the sparsity test),
#            pushes tracked by per-group dirty flags
#   sparse_alld — the same, but every round's commit reads D of every group (no push flags)
#   sparse_direct — every round sparse; with an empty majority the pushes into empty peers go
#            straight into S and the commit recomputes the totals (the heavy-round default)
#   sparse_noq — every round sparse, edges resolved where drawn (scan_queue 0: no per-wave queue)
#   sparse_bscan — every round sparse on the binned scan (edges binned by peer tile, peers tested
#            against an LDS copy of the rare bitmap; bin_scan_frac 0)
#   dense_filter — every round dense, emit dropping edges by the peer's class (occupancy bitmaps)
#   direct — the random-access kernels
PATHS = ["auto", "dense", "dense_filter", "sparse", "sparse_alld", "sparse_direct", "sparse_noq", "sparse_bscan",
         "direct"]
_PATH_FLAGS = {"auto": 0, "dense": FLAG_DENSE, "dense_filter": 0, "sparse": 0, "sparse_alld": 0, "sparse_direct": 0,
               "sparse_noq": 0, "sparse_bscan": 0, "direct": FLAG_DIRECT}
# gossip_set_param knobs; alld_frac: 0 = every sparse round commits every group's D, huge = none does
_PATH_PARAMS = {"dense_filter": {"sparse_frac": -1, "filter_frac": 0},
                "sparse": {"sparse_frac": 1.0, "alld_frac": 1e30},
                "sparse_alld": {"sparse_frac": 1.0, "alld_frac": 0, "sparse_direct": 0},
                "sparse_direct": {"sparse_frac": 1.0, "alld_frac": 0, "sparse_direct": 1},
                "sparse_noq": {"sparse_frac": 1.0, "scan_queue": 0},
                "sparse_bscan": {"sparse_frac": 1.0, "bin_scan_frac": 0}}


@pytest.fixture
def path(request):
    """(flags, params) of one round path"""
    name = request.param
    return _PATH_FLAGS[name], _PATH_PARAMS.get(name, {})


@pytest.mark.parametrize("path", PATHS, indirect=True)
@pytest.mark.parametrize("idx", range(8))
def test_random_golden(golden, idx, path):
    c = golden["random"][idx]
    e = Engine(c["N"], c["R"], c["mode"], c["k"], c["seed"], flags=1 | path[0], params=path[1])
    inject_case(e, c["inject"])
    res = e.step(256)
    assert res.rounds == len(c["rounds"])
    for got, inf, want in zip(res.stats, res.infected, c["rounds"]):
        assert (got["full_nodes"], got["converged"], got["state_hash"]) == (want["full"], want["converged"], want["hash"])
        assert [int(x) for x in inf] == want["infected"]
    assert e.state_hash() == c["final_hash"]


@pytest.mark.parametrize("idx", range(7))
def test_flood_golden(golden, idx):
    c = golden["flood"][idx]
    e = Engine(c["N"], c["R"], "flood", 0, 0, flags=1)
    e.set_topology(c["adj"])
    inject_case(e, c["inject"])
    res = e.step(256)
    assert [s["messages"] for s in res.stats] == [r["messages"] for r in c["rounds"]]
    assert [s["state_hash"] for s in res.stats] == [r["hash"] for r in c["rounds"]]
    for node, want in c["reads"].items():
        assert e.read(int(node)) == want


_ORACLE_CACHE = {}


def _oracle_run(cfg, inj, rounds, threads):
    """Oracle result for cfg, computed once per session and shared by every path."""
    key = (cfg, str(inj), rounds)
    if key not in _ORACLE_CACHE:
        N, R, mode, k, seed = cfg
        o = op.OracleEngine(N, R, mode, k, seed, flags=1, threads=threads)
        inject_case(o, inj)
        ro = o.step(rounds)
        _ORACLE_CACHE.clear()  # keep one state image alive at a time
        _ORACLE_CACHE[key] = (ro, o.read_shard())
    return _ORACLE_CACHE[key]


def _compare(cfg, inj="random", rounds=256, threads=THREADS, path=(0, {})):
    N, R, mode, k, seed = cfg
    e = Engine(N, R, mode, k, seed, flags=1 | path[0], params=path[1])
    inject_case(e, inj)
    re_ = e.step(rounds)
    ro, oshard = _oracle_run(cfg, inj, rounds, threads)
    assert re_.stats == ro.stats
    assert np.array_equal(re_.infected, ro.infected)
    assert np.array_equal(e.read_shard(), oshard)
    return re_


@pytest.mark.parametrize("path", PATHS, indirect=True)
def test_cfg2_push_1M_k3(path):
    """configs[1]: 1M nodes, push fanout 3, one rumor, seed 0x5EED0001."""
    res = _compare((1 << 20, 1, "push", 3, 0x5EED0001), [(0, 0)], path=path)
    assert res.converged and 12 <= res.rounds <= 20


@pytest.mark.parametrize("path", PATHS, indirect=True)
def test_pull_and_multiword(path):
    _compare((1 << 18, 1, "pull", 2, 0x5EED0002), [(123, 0)], path=path)
    _compare((100003, 130, "pushpull", 3, 77), path=path)
    _compare((65536, 64, "push", 1, 5), path=path)
    _compare((300007, 17, "pushpull", 5, 0xFEED), path=path)   # ragged tiles, fanout 5
    _compare((40000, 64, "pull", 9, 0xC0FFEE), path=path)      # fanout > 8: small sender tiles


@pytest.mark.parametrize("path", PATHS, indirect=True)
def test_cfg3_pushpull_16M_r64(path):
    """configs[2]: 16M nodes, push-pull fanout 2, 64 rumors at Philox origins."""
    res = _compare((1 << 24, 64, "pushpull", 2, 0x5EED0003), path=path)
    assert res.converged
    inf = res.infected.astype(np.int64)
    assert (np.diff(inf, axis=0) >= 0).all() and (inf[-1] == 1 << 24).all()


def test_placement_trials_move_time_not_bits():
    """Before its first round a configs[2] engine times trial rounds on fresh allocations of its
    record slab (param place_tries): 12 candidates x 3 rounds in timer 5 by default,
    none with place_tries 1; the rounds equal the oracle's either way."""
    cfg = (1 << 24, 64, "pushpull", 2, 0x5EED0003)
    ro, oshard = _oracle_run(cfg, "random", 256, THREADS)
    for params, trials in (({}, 36), ({"place_tries": 1}, 0)):
        e = Engine(*cfg, flags=1 | FLAG_TIMING, params=params)
        inject_case(e, "random")
        r = e.step(256)
        assert r.stats == ro.stats and np.array_equal(r.infected, ro.infected)
        assert np.array_equal(e.read_shard(), oshard)
        assert e.kernel_time(5)[1] == trials
        e.close()


@pytest.mark.parametrize("path", PATHS, indirect=True)
def test_tiny_and_edge_sizes(path):
    _compare((2, 1, "pushpull", 2, 1), [(1, 0)], path=path)
    _compare((3, 64, "push", 4, 9), path=path)
    _compare((1000, 1, "pull", 1, 3), [(999, 0)], path=path)
    _compare((16385, 64, "pushpull", 64, 3), path=path)  # maximum fanout, one-node last tile
    # no injection: nothing ever spreads, never converges
    e = Engine(5000, 1, "pushpull", 2, 1)
    res = e.step(5)
    assert res.rounds == 5 and not res.converged and res.infected.sum() == 0


@pytest.mark.parametrize("path", PATHS, indirect=True)
def test_inject_between_steps(path):
    """A client broadcast between rounds (main.go:102-117) invalidates the
    engine's running totals and occupancy bitmaps; the next round rebuilds them."""
    cfg = (200003, 11, "pushpull", 2, 0x5EED0007)
    e = Engine(*cfg, flags=1 | path[0], params=path[1])
    o = op.OracleEngine(*cfg, flags=1, threads=THREADS)
    for x in (e, o):
        x.inject(5, 0)
        x.inject(77777, 10)
    for burst in ([(123, 1), (5, 2)], [(200002, 3), (9, 4)], [(0, 5), (1, 6), (2, 7), (3, 8), (4, 9)]):
        a, b = e.step(3), o.step(3)
        assert a.stats == b.stats and np.array_equal(a.infected, b.infected)
        for x in (e, o):
            for n, r in burst:
                x.inject(n, r)
    a, b = e.step(200), o.step(200)
    assert a.stats == b.stats and a.converged
    assert np.array_equal(e.read_shard(), o.read_shard())


def test_reset_and_rerun_identical():
    e = Engine(1 << 16, 64, "pushpull", 2, 21, flags=1)
    e.inject_random()
    a = e.step(100)
    e.reset()
    e.inject_random()
    b = e.step(100)
    assert a.stats == b.stats


def test_maelstrom_cluster_grid25():
    c = Cluster(25, max_values=3)
    c.topology(grid_topology(25))
    c.broadcast("n0", 1000)
    c.broadcast("n24", -7)
    c.broadcast("n0", 1000)  # dedupe, main.go:113
    res = c.gossip()
    # both values are everywhere after 8 rounds; the last learners still forward
    # once (round 8) and round 9 sends nothing (quiescence stop)
    assert res.rounds == 10 and res.stats[-1]["messages"] == 0
    assert [int(x) for x in res.infected[7][:2]] == [25, 25]
    for i in range(25):
        assert sorted(c.read(f"n{i}")) == [-7, 1000]


def test_errors():
    e = Engine(100, 2, "flood", 0, 0)
    with pytest.raises(GossipError) as ei:
        e.step(3)
    assert ei.value.code == -4  # ESTATE: FLOOD without topology
    with pytest.raises(GossipError):
        e.inject(100, 0)
    with pytest.raises(GossipError):
        e.inject(0, 2)
    with pytest.raises(GossipError):
        e.set_topology(([0, 1], [0]))  # wrong node count


def _dev_tensor(ptr, nbytes):
    from gossip_hip.sharded import _as_tensor
    return _as_tensor(ptr, nbytes, True)


@pytest.mark.parametrize("mode,k,R,N", [("pushpull", 2, 64, 300001), ("push", 3, 1, 1 << 18),
                                         ("pull", 2, 130, 50000), ("flood", 0, 2, 400)])
def test_two_shards_on_one_gpu(mode, k, R, N):
    """The sharded round protocol with both shards on one device: the all-gather
    is done with device copies; results equal the unsharded engine bit for bit."""
    seed = 0x5EED0004
    shards = [Engine(N, R, mode, k, seed, flags=1, shard_rank=r, shard_count=2) for r in range(2)]
    ref = Engine(N, R, mode, k, seed, flags=1)
    engines = shards + [ref]
    if mode == "flood":
        adj = [[int(v[1:]) for v in grid_topology(N)[f"n{i}"]] for i in range(N)]
        for e in engines:
            e.set_topology(adj)
            e.inject(0, 0)
            e.inject(N - 1, 1)
    else:
        for e in engines:
            e.inject_random()
    want = ref.step(200)
    got = []
    for _ in range(200):
        bufs = [s.exchange_buffers() for s in shards]
        nbytes = bufs[0][2]
        for r, s in enumerate(shards):  # all-gather: every shard's slice into every image
            dst = _dev_tensor(bufs[r][1], nbytes * 2)
            for q in range(2):
                dst[q * (nbytes // 8):(q + 1) * (nbytes // 8)].copy_(_dev_tensor(bufs[q][0], nbytes))
        torch.cuda.synchronize()
        parts = [s.round_compute() for s in shards]
        total = parts[0] + parts[1]
        st = [s.round_commit(total) for s in shards]
        assert st[0] == st[1]
        got.append(st[0])
        if st[0]["converged"] or (mode == "flood" and st[0]["messages"] == 0):
            break
    assert got == want.stats
    full = ref.read_shard()
    for s in shards:
        assert np.array_equal(s.read_shard(), full[:, s.lo:s.hi])


@pytest.mark.parametrize("idx", range(3))
def test_antientropy_golden_gpu(golden, idx):
    c = golden["antientropy"][idx]
    e = Engine(c["N"], c["K"], "antientropy", c["k"], c["seed"], flags=1,
               churn_fail=c["fail"], churn_recover=c["recover"])
    e.inject_random()
    e.inject(c["N"] - 1, 0)
    res = e.step(300)
    assert res.rounds == len(c["rounds"])
    for got, inf, want in zip(res.stats, res.infected, c["rounds"]):
        assert (got["full_nodes"], got["alive_nodes"], got["messages"], got["state_hash"], got["converged"]) == \
            (want["full"], want["alive"], want["messages"], want["hash"], want["converged"])
        assert [int(x) for x in inf] == want["infected"]
    v, alive = e.read_versions(0)
    assert [int(x) for x in v] == c["node0"] and alive == c["node0_alive"]


def test_antientropy_vs_oracle_1M():
    from gossip_hip.engine import churn_threshold as ct
    N, K, k, seed = 1 << 20, 16, 1, 0x5EED0005
    e = Engine(N, K, "antientropy", k, seed, flags=1, churn_fail=ct(0.01), churn_recover=ct(0.1))
    o = op.OracleEngine(N, K, "antientropy", k, seed, flags=1, churn_fail=ct(0.01), churn_recover=ct(0.1))
    for x in (e, o):
        x.inject_random()
    a, b = e.step(200), o.step(200)
    assert a.stats == b.stats and np.array_equal(a.infected, b.infected)
    assert a.converged
    for node in (0, 1, N // 3, N - 1):
        assert [int(x) for x in e.read_versions(node)[0]] == [int(x) for x in o.read_versions(node)[0]]


def test_antientropy_cfg5_64M_properties():
    """configs[4] at full size: 2^26 nodes, K=16, fanout 1, churn 1% / 10%."""
    from gossip_hip.engine import churn_threshold as ct
    N = 1 << 26
    e = Engine(N, 16, "antientropy", 1, 0x5EED0005, churn_fail=ct(0.01), churn_recover=ct(0.1))
    e.inject_random()
    res = e.step(400)
    # convergence waits for the stale nodes that died before the versions reached
    # them: they revive at 10% per round, so ~log(0.6M)/log(1/0.9) ~ 126 rounds
    assert res.converged and res.rounds < 300
    inf = res.infected.astype(np.int64)
    alive = np.array([s["alive_nodes"] for s in res.stats])
    assert (inf <= alive[:, None]).all()
    # steady-state alive fraction of the churn chain is 0.1 / 0.11
    assert 0.85 * N < alive[-1] <= N
