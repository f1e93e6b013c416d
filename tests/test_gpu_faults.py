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
         "sparse_alld": (0, {"sparse_frac": 1.0, "alld_frac": 0, "sparse_direct": 0}),
         "sparse_direct": (0, {"sparse_frac": 1.0, "alld_frac": 0}), "direct": (FLAG_DIRECT, {})}


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


# --- stall mode and FLOOD retries, against the numpy goldens -------------------

@pytest.mark.parametrize("path", list(PATHS))
@pytest.mark.parametrize("idx", range(5))
def test_random_faults_stall_golden_every_path(golden, idx, path):
    """Edge loss / partitions and the stall mode on every round path (auto, dense, dense with the
    peer-class filter, sparse, sparse all-D, direct) equal the numpy restatement round by round."""
    from conftest import inject_case
    c = golden["random_faults"][idx]
    flags, params = PATHS[path]
    e = Engine(c["N"], c["R"], c["mode"], c["k"], c["seed"], flags=1 | flags, edge_loss=c["edge_loss"],
               partitions=c["partitions"], stall_rounds=c["stall_rounds"], params=params)
    inject_case(e, c["inject"])
    res = e.step(c["max_rounds"])
    assert res.rounds == len(c["rounds"])
    for got, inf, want in zip(res.stats, res.infected, c["rounds"]):
        assert (got["full_nodes"], got["converged"], got["state_hash"]) == (want["full"], want["converged"], want["hash"])
        assert [int(x) for x in inf] == want["infected"]
    assert e.state_hash() == c["final_hash"]
    e.close()


def _n_flood_faults():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.json")) as f:
        return len(json.load(f)["flood_faults"])


@pytest.mark.parametrize("idx", range(_n_flood_faults()))
def test_flood_faults_golden_gpu(golden, idx):
    """FLOOD with per-edge retries and the deadline stall (round_flood_faults_kernel)."""
    from conftest import inject_case
    c = golden["flood_faults"][idx]
    e = Engine(c["N"], c["R"], "flood", 0, 0, flags=1, edge_loss=c["edge_loss"], partitions=c["partitions"],
               stall_rounds=c["stall_rounds"])
    e.set_topology(c["adj"])
    inject_case(e, c["inject"])
    res = e.step(c["max_rounds"])
    assert [s["messages"] for s in res.stats] == [r["messages"] for r in c["rounds"]]
    assert [s["state_hash"] for s in res.stats] == [r["hash"] for r in c["rounds"]]
    assert [s["full_nodes"] for s in res.stats] == [r["full"] for r in c["rounds"]]
    for node, want in c["reads"].items():
        assert e.read(int(node)) == want


@pytest.mark.parametrize("idx", range(7))
def test_flood_edge_kernel_without_losses_equals_flood_gpu(golden, idx):
    """The FLOOD walk kernel with nothing lost reproduces the fault-free goldens (rows without
    repeated entries: the walks send to each entry, plain FLOOD reads rows as sets)."""
    from conftest import inject_case
    c = golden["flood"][idx]
    if any(len(set(r)) != len(r) for r in c["adj"]):
        pytest.skip("repeated row entries: the walks send to each entry")
    e = Engine(c["N"], c["R"], "flood", 0, 0, flags=1, stall_rounds=1)
    e.set_topology(c["adj"])
    inject_case(e, c["inject"])
    res = e.step(256)
    assert [s["messages"] for s in res.stats] == [r["messages"] for r in c["rounds"]]
    assert [s["state_hash"] for s in res.stats] == [r["hash"] for r in c["rounds"]]


@pytest.mark.parametrize("path", list(PATHS))
def test_stall_streaks_across_steps_and_injects(path):
    """Stall streaks carry across gossip_step calls (short steps, injects between them, a step
    after convergence) exactly as the oracle carries them: the pipelined step runs no round
    ahead of the one it waits on when streaks are kept (stall_d is not idempotent)."""
    N, R, k, seed, loss, D = 3001, 6, 2, 0x5EED0009, loss_threshold(0.05), 2
    flags, params = PATHS[path]
    e = Engine(N, R, "pushpull", k, seed, flags=1 | flags, edge_loss=loss, stall_rounds=D, params=params)
    o = op.OracleEngine(N, R, "pushpull", k, seed, flags=1, edge_loss=loss, stall_rounds=D)
    for x in (e, o):
        x.inject(5, 0)
        x.inject(N - 1, 1)
    for burst in ([(123, 2)], [(7, 3), (2999, 4)], [(0, 5)]):
        a, b = e.step(3), o.step(3)
        assert a.stats == b.stats and np.array_equal(a.infected, b.infected)
        for x in (e, o):
            for n, r in burst:
                x.inject(n, r)
    a, b = e.step(300), o.step(300)
    assert a.stats == b.stats and a.converged
    a, b = e.step(5), o.step(5)  # past convergence: nothing moves, the round counters agree
    assert a.stats == b.stats
    assert np.array_equal(e.read_shard(), o.read_shard())
    e.close()


@pytest.mark.parametrize("plan", ["auto", "sparse", "dense"])
def test_stall_sharded_lockstep(plan):
    """Stall streaks are kept for all N nodes on every shard: G = 3 lockstep equals the oracle."""
    N, R, k, seed, loss, D = 30011, 64, 2, 0x5EED0004, loss_threshold(0.1), 3
    ref = op.OracleEngine(N, R, "pushpull", k, seed, flags=1, edge_loss=loss, stall_rounds=D)
    ref.inject_random()
    want, full = ref.step(200), ref.read_shard()
    params = {} if plan == "auto" else {"sparse_frac": 1.0 if plan == "sparse" else -1}
    engines = [Engine(N, R, "pushpull", k, seed, flags=1, shard_rank=r, shard_count=3, edge_loss=loss,
                      stall_rounds=D, params=params) for r in range(3)]
    for e in engines:
        e.inject_random()
    got, _ = lockstep_run(engines, 200)
    assert got == want.stats
    for e in engines:
        assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])
        e.close()


def test_flood_walks_topology_change_mid_run_gpu():
    """A topology message mid-run ends every walk (a known divergence from
    main.go:72, whose goroutine keeps the row it read): the GPU equals the oracle round by round,
    before and after the change, with losses and the deadline stall."""
    N, R = 30, 3
    row_a = [[(u + 1) % N, (u + 7) % N] for u in range(N)]
    row_b = [[(u + 3) % N, (u + 11) % N, (u + 1) % N] for u in range(N)]
    kw = dict(edge_loss=loss_threshold(0.3), stall_rounds=2)
    runs = []
    for x in (Engine(N, R, "flood", 0, 5, flags=1, **kw), op.OracleEngine(N, R, "flood", 0, 5, flags=1, **kw)):
        x.set_topology(row_a)
        for r in range(R):
            x.inject(r * 9, r)
        a = x.step(3)
        x.set_topology(row_b)
        x.inject(4, 0)
        b = x.step(60)
        runs.append((a.stats, b.stats, x.read_shard()))
        x.close()
    assert runs[0][0] == runs[1][0] and runs[0][1] == runs[1][1]
    assert np.array_equal(runs[0][2], runs[1][2])
