"""GPU parity of the ANTIENTROPY round paths against the CPU oracle,
bit-exact per round: stats, per-component counts, hash, and the rows and alive flags read back.

Paths (all must agree with the oracle and with each other):
  auto     — dense rounds until the stale nodes are few, then sparse in-place rounds
  dense    — ae_sparse = 0: every round dense (binned in-edge gathers, stats fused; once the stale
             bits are exact, exchanges that cannot move a row are skipped: the stale filter)
  dense_nofilter — ae_dense_filter = 0: binned dense rounds gather every exchange's rows
  dense_atomic — ae_dense_bin = 0: dense rounds as pull pass + atomicMax push pass + stats pass
  dense_ranges — ae_dense_cap = 256: each tile's in-edges sorted in many LDS passes
  dense_fallback — ae_dense_cap = 16: every binned dense round overflows and is rerun atomically
  sparse   — ae_sparse = 1: every round after the first sparse (the edge list holds k*N)
  overflow — sparse forced with a 64-edge list (ae_cap): rounds whose list overflows are rerun dense
  *_direct — FLAG_AE_DIRECT_SCAN: the sparse scan probes the peers' bitmap words directly
             instead of binning the exchanges by the peer's tile
  Runs of sparse rounds are pipelined (engine step_ae: ae_ahead rounds enqueued at once, each gated
  on device by its predecessor); *_ahead1 runs them one at a time, *_ahead3 three at a time.
"""
import os

import numpy as np
import pytest

import oracle_py as op
from gossip_hip import FLAG_AE_DIRECT_SCAN, Engine
from gossip_hip.engine import churn_threshold as ct

pytestmark = pytest.mark.gpu
THREADS = min(16, os.cpu_count() or 1)
# (flags, gossip_set_param knobs) per path
PATHS = {"auto": (0, {}), "dense": (0, {"ae_sparse": 0}), "sparse": (0, {"ae_sparse": 1}),
         "dense_atomic": (0, {"ae_sparse": 0, "ae_dense_bin": 0}),
         "dense_nofilter": (0, {"ae_sparse": 0, "ae_dense_filter": 0}),
         "dense_ranges": (0, {"ae_sparse": 0, "ae_dense_cap": 256}),
         "dense_fallback": (0, {"ae_sparse": 0, "ae_dense_cap": 16}),
         "overflow": (0, {"ae_sparse": 1, "ae_cap": 64}),
         # sparse rounds with the direct scan (random bitmap probes) instead of the binned one
         "sparse_direct": (FLAG_AE_DIRECT_SCAN, {"ae_sparse": 1}),
         "auto_direct": (FLAG_AE_DIRECT_SCAN, {}),
         "auto_ahead1": (0, {"ae_ahead": 1}), "sparse_ahead3": (0, {"ae_sparse": 1, "ae_ahead": 3}),
         "overflow_ahead3": (0, {"ae_sparse": 1, "ae_cap": 64, "ae_ahead": 3})}


def _engine(path, *args, flags=0, **kw):
    pf, params = PATHS[path]
    return Engine(*args, flags=flags | pf, params=params, **kw)


def _compare(e, o, N, K, rounds, probe):
    a, b = e.step(rounds), o.step(rounds)
    assert a.rounds == b.rounds
    assert a.stats == b.stats
    assert np.array_equal(a.infected, b.infected)
    for node in probe:
        (ve, ae), (vo, ao) = e.read_versions(node), o.read_versions(node)
        assert np.array_equal(ve, vo) and ae == ao, node
    assert e.state_hash() == o.state_hash()
    return a


@pytest.mark.parametrize("path", list(PATHS))
@pytest.mark.parametrize("N,K,k,fail,rec", [
    (1 << 16, 16, 1, 0.01, 0.1),
    (50_001, 5, 2, 0.05, 0.3),
    (4099, 64, 3, 0.02, 0.2),
    (777, 1, 1, 0.0, 0.0),
])
def test_antientropy_paths_vs_oracle(path, N, K, k, fail, rec):
    seed = 0x5EED0005 + K
    kw = dict(flags=1, churn_fail=ct(fail), churn_recover=ct(rec))
    e = _engine(path, N, K, "antientropy", k, seed, **kw)
    o = op.OracleEngine(N, K, "antientropy", k, seed, threads=THREADS, **kw)
    probe = (0, 1, N // 3, N // 2, N - 1)
    for x in (e, o):
        x.inject_random()
    _compare(e, o, N, K, 6, probe)           # a few rounds, then a client write mid-run
    for x in (e, o):
        x.inject(N // 2, K - 1)
        x.inject(3, 0)
    res = _compare(e, o, N, K, 400, probe)
    assert res.converged


def test_antientropy_sparse_tail_1M():
    """configs[4] shape at 2^20: the churn tail runs sparse (auto) and matches the oracle."""
    N, K, k, seed = 1 << 20, 16, 1, 0x5EED0005
    kw = dict(flags=1, churn_fail=ct(0.01), churn_recover=ct(0.1))
    e = _engine("auto", N, K, "antientropy", k, seed, **kw)
    o = op.OracleEngine(N, K, "antientropy", k, seed, threads=THREADS, **kw)
    for x in (e, o):
        x.inject_random()
    res = _compare(e, o, N, K, 300, (0, 7, N // 5, N - 2))
    assert res.converged and res.rounds > 40


def test_reset_zeroes_rows_lazily():
    """gossip_reset leaves the zeroing of the rows pending until a call needs it, and
    inject_random (which writes every row) drops it: a read after a reset sees
    zeros, and runs after reset + inject_random, with or without a read in between, equal the
    oracle's.  2^23 rows of K = 16 are 512 MiB, so the rows' placement trials (ae_place) run too."""
    N, K, k, seed = 1 << 23, 16, 1, 0x5EED0005
    kw = dict(flags=1, churn_fail=ct(0.01), churn_recover=ct(0.1))
    e = _engine("auto", N, K, "antientropy", k, seed, **kw)
    o = op.OracleEngine(N, K, "antientropy", k, seed, threads=THREADS, **kw)
    for x in (e, o):
        x.inject_random()
    _compare(e, o, N, K, 3, (0, N - 1))
    e.reset()
    assert not e.read_rows().any()           # the pending zeroing ran before the read
    for x in (e, o):
        x.reset()
        x.inject_random()
    _compare(e, o, N, K, 4, (0, 5, N - 1))
    for x in (e, o):                          # reset straight into a random write: no zeroing at all
        x.reset()
        x.inject_random()
    res = _compare(e, o, N, K, 400, (1, N // 2, N - 1))
    assert res.converged


def test_dense_bin_params():
    """The binned dense round's knobs are validated; K > 16 engines keep the atomic passes."""
    e = Engine(4096, 16, "antientropy", 1, 0x5EED0005, flags=1, params={"ae_dense_bin": 1, "ae_dense_cap": 0})
    for name, bad in (("ae_dense_bin", 2), ("ae_dense_bin", -1), ("ae_dense_cap", -1), ("ae_dense_cap", 70000)):
        with pytest.raises(Exception):
            e.set_param(name, bad)
    e.set_param("ae_dense_bin", 0)
    e.set_param("ae_dense_cap", 64)


def test_init_target_K12_past_grid_stride():
    """K = 12 (3 quads per row) past ~5.6M nodes: ae_init_kernel's grid stride (2^24 threads) is no
    multiple of 3, so a thread's quad changes between iterations and its running maxima must be
    flushed per quad.  The target and the first rounds equal the oracle's."""
    N, K, k, seed = (1 << 23) + 77, 12, 1, 0x5EED000C
    kw = dict(flags=1, churn_fail=ct(0.01), churn_recover=ct(0.1))
    e = _engine("auto", N, K, "antientropy", k, seed, **kw)
    o = op.OracleEngine(N, K, "antientropy", k, seed, threads=THREADS, **kw)
    for x in (e, o):
        x.inject_random()
    _compare(e, o, N, K, 4, (0, 1, N // 3, N - 1))
