"""GPU: G shard engines on one device, driven in lockstep through the sharded
round protocol (include/gossip.h) with device copies standing in
for the RCCL collectives, equal a single-engine run bit for bit — per-round
stats, per-rumor counts and the final state.  Sparse rounds (rare-list
all-gather + push all-to-all) and dense rounds (state all-gather) are forced
one at a time and mixed as the engines plan them."""
import numpy as np
import pytest
import torch

from gossip_hip import FLAG_SHARD_DIRECT, Engine
from gossip_hip.sharded import lockstep_run as run_lockstep

pytestmark = pytest.mark.gpu


CASES = [("pushpull", 2, 64, 1 << 20, 0x5EED0004, 4), ("push", 3, 1, 300001, 7, 3),
         ("pull", 1, 5, 100000, 11, 2), ("pushpull", 6, 7, 50001, 3, 2),
         # tiny clusters whose last shard owns no node (3, 3, 3, 3, 0 and 3, 3, 3, 0)
         ("pushpull", 2, 5, 12, 3, 5), ("push", 1, 1, 9, 5, 4)]
IDS = ["pushpull-1M-G4", "push-ragged-G3", "pull-G2", "pushpull-k6-G2", "pushpull-N12-G5-empty", "push-N9-G4-empty"]
# (flags, gossip_set_param knobs) per plan
PLANS = {"auto": (0, {}), "sparse": (0, {"sparse_frac": 1.0}), "sparse_alld": (0, {"sparse_frac": 1.0, "alld_frac": 0}),
         "dense": (0, {"sparse_frac": -1, "xd_shards": 0, "cc_frac": 0}),
         # the state all-gather class-coded (bitmaps + mixed words)
         "classcoded": (0, {"sparse_frac": -1, "xd_shards": 0, "cc_frac": 1}),
         # dense rounds as exchange rounds (items to the peer's owner, replies back)
         "exchange": (0, {"sparse_frac": -1, "xd_shards": 2}), "auto_exchange": (0, {"xd_shards": 2}),
         # exchange rounds that never drop edges by the peer's class (filter_frac 1)
         "exchange_unfiltered": (0, {"sparse_frac": -1, "xd_shards": 2, "xd_filter_frac": 1.0}),
         # dense sharded rounds on the direct kernels instead of the binned push/pull passes
         "dense_direct": (FLAG_SHARD_DIRECT, {"sparse_frac": -1, "xd_shards": 0, "cc_frac": 0}),
         "classcoded_direct": (FLAG_SHARD_DIRECT, {"sparse_frac": -1, "xd_shards": 0, "cc_frac": 1}),
         "auto_direct": (FLAG_SHARD_DIRECT, {"xd_shards": 0}),
         # dense rounds replicated: every shard computes the whole image (kinds 5 / 6)
         "replicated": (0, {"sparse_frac": -1, "replicate": 1}), "auto_replicated": (0, {"replicate": 1})}


@pytest.mark.parametrize("plan", list(PLANS))
@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_lockstep_shards_equal_one_engine(case, plan):
    mode, k, R, N, seed, G = case
    ref = Engine(N, R, mode, k, seed, flags=1)
    ref.inject_random()
    want = ref.step(200)
    full = ref.read_shard()
    ref.close()
    flags, params = PLANS[plan]
    engines = [Engine(N, R, mode, k, seed, flags=1 | flags, shard_rank=r, shard_count=G, params=params)
               for r in range(G)]
    for e in engines:
        e.inject_random()
    got, kinds = run_lockstep(engines, 200)
    assert got == want.stats
    for e in engines:
        assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])
    if plan in ("sparse", "sparse_alld"):
        assert set(kinds) == {1}
    elif plan in ("dense", "dense_direct"):
        assert set(kinds) == {0}
    elif plan in ("exchange", "exchange_unfiltered"):
        assert set(kinds) == {3}
    elif plan in ("classcoded", "classcoded_direct"):
        assert set(kinds) == {4}
    elif plan in ("auto", "auto_direct"):
        assert 4 in kinds  # G < xd_shards: dense rounds with few mixed nodes go class-coded
    elif plan == "replicated":  # the image gathered once (whole or class-coded), then whole after every round
        assert kinds[0] in (5, 7) and set(kinds[1:]) <= {6}
    elif plan == "auto_replicated":
        assert set(kinds) & {5, 7} and set(kinds) <= {1, 5, 6, 7}
    for e in engines:
        e.close()


@pytest.mark.parametrize("G", [2, 3])
def test_lockstep_model_replicates_past_2p22(G):
    """Past 2^22 nodes at G = 2-3 the link-aware model prices a replicated dense round (the one-GPU
    round over the whole image, no collective once the image is whole) below the state all-gather
    round, and plans it by itself: kind 5 or 7 (entered over the whole or the class-coded
    all-gather), then 6; the rounds still equal one engine."""
    N, R, k, seed = (1 << 23) + 5, 64, 2, 0x5EED0004
    ref = Engine(N, R, "pushpull", k, seed, flags=1)
    ref.inject_random()
    want = ref.step(200)
    full = ref.read_shard()
    ref.close()
    engines = [Engine(N, R, "pushpull", k, seed, flags=1, shard_rank=r, shard_count=G) for r in range(G)]
    for e in engines:
        e.inject_random()
    got, kinds = run_lockstep(engines, 200)
    assert got == want.stats
    for e in engines:
        assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])
    assert set(kinds) & {5, 7} and 6 in kinds, kinds
    for e in engines:
        e.close()


def test_lockstep_replicated_faults_stall():
    """Replicated rounds draw, lose and stall edges as every other path."""
    from gossip_hip.engine import loss_threshold
    N, R, k, seed, G = 30011, 64, 2, 0x5EED0004, 3
    kw = dict(edge_loss=loss_threshold(0.1), partitions=3, stall_rounds=3)
    ref = Engine(N, R, "pushpull", k, seed, flags=1, **kw)
    ref.inject_random()
    want = ref.step(300)
    full = ref.read_shard()
    ref.close()
    engines = [Engine(N, R, "pushpull", k, seed, flags=1, shard_rank=r, shard_count=G, params={"replicate": 1, "sparse_frac": -1}, **kw)
               for r in range(G)]
    for e in engines:
        e.inject_random()
    got, kinds = run_lockstep(engines, 300)
    assert got == want.stats
    for e in engines:
        assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])
    assert kinds[0] in (5, 7) and set(kinds[1:]) <= {6}
    for e in engines:
        e.close()


def test_lockstep_inject_between_steps():
    """Client broadcasts between runs invalidate the global totals; the next plan re-derives them."""
    N, R, G = 200003, 11, 2
    ref = Engine(N, R, "pushpull", 2, 5, flags=1)
    engines = [Engine(N, R, "pushpull", 2, 5, flags=1, shard_rank=r, shard_count=G) for r in range(G)]
    outs_ref, outs = [], []
    for node, rumor in [(17, 0), (N - 1, 3), (N // 2, 10)]:
        ref.inject(node, rumor)
        for e in engines:
            e.inject(node, rumor)
        outs_ref.append(ref.step(5).stats)
        outs.append(run_lockstep(engines, 5)[0])
    assert outs == outs_ref
    full = ref.read_shard()
    for e in engines:
        assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])


def test_lockstep_dense_past_4096_tiles():
    """Above 2^26 nodes the pull pass of a dense sharded round bins into more than 4096
    image tiles (binned.h: kSbMaxTiles); odd shard size, so every slice but the first
    starts 8-B aligned.  Reference: one engine (direct kernels at this size)."""
    N, R, G = (1 << 26) + 12345, 64, 2
    ref = Engine(N, R, "pushpull", 2, 0x5EED0004, flags=1)
    ref.inject_random()
    want = ref.step(8)
    full = ref.read_shard()
    ref.close()
    for plan, kind in (({"sparse_frac": -1, "xd_shards": 0, "cc_frac": 0}, 0), ({"sparse_frac": -1, "xd_shards": 2}, 3),
                       ({"sparse_frac": -1, "xd_shards": 0, "cc_frac": 1}, 4)):
        engines = [Engine(N, R, "pushpull", 2, 0x5EED0004, flags=1, shard_rank=r, shard_count=G, params=plan)
                   for r in range(G)]
        for e in engines:
            e.inject_random()
        got, kinds = run_lockstep(engines, 8)
        assert got == want.stats and set(kinds) == {kind}
        for e in engines:
            assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])
            e.close()


@pytest.mark.parametrize("k,faults", [(3, {}), (2, dict(edge_loss=1 << 29, partitions=3))], ids=["k3", "k2-faults"])
def test_lockstep_dense_past_4096_tiles_big_regions(k, faults):
    """Past 4096 image tiles the sharded dense round's passes take 16384-sender regions
    (make_sb_geom; binned.hip emit V = 6, 7 with redrawn peers for k > 2 or faults; k <= 2
    without faults keeps them, V = 8, 9: test_lockstep_dense_past_4096_tiles).  Two ragged shards
    on the state all-gather, every round dense, against one engine."""
    N, R, G = (1 << 26) + 12345, 64, 2
    ref = Engine(N, R, "pushpull", k, 0x5EED0007, flags=1, **faults)
    ref.inject_random()
    want = ref.step(6)
    full = ref.read_shard()
    ref.close()
    engines = [Engine(N, R, "pushpull", k, 0x5EED0007, flags=1, shard_rank=r, shard_count=G,
                      params={"sparse_frac": -1, "xd_shards": 0, "cc_frac": 0}, **faults) for r in range(G)]
    for e in engines:
        e.inject_random()
    got, kinds = run_lockstep(engines, 6)
    assert got == want.stats and set(kinds) == {0}
    for e in engines:
        assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])
        e.close()


@pytest.mark.parametrize("plan", [({"xd_shards": 2, "sparse_frac": -1}, 3),
                                  ({"xd_shards": 0, "sparse_frac": -1, "cc_frac": 1}, 4)], ids=["exchange", "classcoded"])
@pytest.mark.parametrize("faults", [dict(edge_loss=1 << 29, partitions=3), dict(edge_loss=1 << 29, stall_rounds=2),
                                    dict(edge_loss=1 << 30, partitions=2, stall_rounds=3)],
                         ids=["loss-partitions", "loss-stall", "all"])
def test_lockstep_exchange_faults_stall(faults, plan):
    """Exchange dense rounds and class-coded all-gathers (every round) with edge loss,
    partitions and the stall mode, G = 5 ragged shards, against one engine."""
    N, R, G = 400009, 64, 5
    ref = Engine(N, R, "pushpull", 2, 0x5EED0006, flags=1, **faults)
    ref.inject_random()
    want = ref.step(60)
    full = ref.read_shard()
    ref.close()
    engines = [Engine(N, R, "pushpull", 2, 0x5EED0006, flags=1, shard_rank=r, shard_count=G,
                      params=plan[0], **faults) for r in range(G)]
    for e in engines:
        e.inject_random()
    got, kinds = run_lockstep(engines, 60)
    assert got == want.stats and set(kinds) == {plan[1]}
    for e in engines:
        assert np.array_equal(e.read_shard(), full[:, e.lo:e.hi])
        e.close()



@pytest.mark.parametrize("filter_frac", [0.3, 1.0], ids=["filtered", "unfiltered"])
def test_exchange_items_equal_oracle(filter_frac):
    """Every round an exchange round at G = 3: the items each shard sends to each owner (after
    the class filter of DESIGN.md §5.2 in the rounds where it applies) are the oracle's, count for
    count, round for round, and so are the stats; the filtered run sends fewer items."""
    import oracle_py as op
    N, G, R, k, seed = 200003, 3, 64, 2, 0x5EED0004
    params = {"sparse_frac": -1, "xd_shards": 2, "xd_filter_frac": filter_frac}
    runs = []
    for mk in (lambda r: Engine(N, R, "pushpull", k, seed, flags=1, shard_rank=r, shard_count=G, params=params),
               lambda r: op.OracleEngine(N, R, "pushpull", k, seed, flags=1, shard_rank=r, shard_count=G,
                                         params=params)):
        engines = [mk(r) for r in range(G)]
        for e in engines:
            e.inject_random()
        items = []
        stats, kinds = run_lockstep(engines, 200, items=items)
        assert set(kinds) == {3}
        runs.append((stats, items))
        if engines[0].on_device:
            for e in engines:
                e.close()
    (hs, hi), (os_, oi) = runs
    assert hs == os_ and hi == oi
    sent = sum(sum(map(sum, r)) for r in hi)
    if filter_frac < 1:  # unfiltered, every round sends k items per node (no node is empty and full)
        assert sent < 0.8 * k * N * len(hi)
