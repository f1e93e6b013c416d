"""GPU, the one-shard round paths past 2^25 nodes against the OpenMP oracle.

Past 2^25 nodes the occupancy bitmaps outgrow an XCD's L2, so sparse rounds test a peer in an
L2-resident mid-level summary before its exact bitmap word (FrontierBufs::summ2,
csrc/frontier.hip); and every heavy sparse round with an empty majority ORs the pushes into
empty peers straight into the state (kSparseDirect).  Every round on the dense pipeline (big
regions, packed pushes) is here too.  Each path must equal the oracle bit for
bit: per-round stats, per-rumor counts and the final state.  Ragged N (not a multiple of 64 or
of the summary groups).  Reference: (*NodeState).Gossip, main.go:65-89, as rounds.
"""
import os

import numpy as np
import pytest

import oracle_py as op
from gossip_hip import Engine

pytestmark = pytest.mark.gpu

N = (1 << 25) + 4099
THREADS = min(16, os.cpu_count() or 1)
# sparse_flags: every round sparse, pushes tracked by dirty flags; sparse_alld: commits read all
# of D; sparse_direct: pushes into empty peers go to S (empty-majority rounds); sparse_mid: every
# round tests summary hits in the mid-level summary (mid_frac 0); auto: as planned
PATHS = {"auto": {}, "sparse_flags": {"sparse_frac": 1.0, "alld_frac": 1e30},
         "sparse_alld": {"sparse_frac": 1.0, "alld_frac": 0, "sparse_direct": 0},
         "sparse_direct": {"sparse_frac": 1.0, "alld_frac": 0, "sparse_direct": 1},
         "sparse_mid": {"sparse_frac": 1.0, "mid_frac": 0},
         # edges resolved where they are drawn (no per-wave queue; the default before round 5)
         "sparse_noq": {"sparse_frac": 1.0, "scan_queue": 0},
         # every round on the binned scan (round 6), with the heavy rounds' direct commits and
         # with dirty flags throughout
         "sparse_bscan": {"sparse_frac": 1.0, "bin_scan_frac": 0},
         "sparse_bscan_flags": {"sparse_frac": 1.0, "bin_scan_frac": 0, "alld_frac": 1e30},
         # every round on the dense pipeline (16384-sender regions, packed pushes)
         "dense": {"sparse_frac": -1.0}}
CASES = {"pushpull-k2-R64": ("pushpull", 2, 64, 0x5EED0003, 0), "push-k3-R5": ("push", 3, 5, 77, 0),
         "pull-k1-R7-loss": ("pull", 1, 7, 9, 1 << 30), "pull-k2-R3": ("pull", 2, 3, 0x51, 0)}


@pytest.fixture(scope="module")
def oracle_runs():
    cache = {}

    def get(case):
        if case not in cache:
            mode, k, r, seed, loss = CASES[case]
            o = op.OracleEngine(N, r, mode, k, seed, flags=1, threads=THREADS, edge_loss=loss)
            o.inject_random()
            res = o.step(200)
            cache[case] = (res, o.read_shard())
            o.close()
        return cache[case]
    return get


@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("path", list(PATHS))
def test_big_paths_equal_oracle(oracle_runs, case, path):
    mode, k, r, seed, loss = CASES[case]
    ro, full = oracle_runs(case)
    e = Engine(N, r, mode, k, seed, flags=1, edge_loss=loss, params=PATHS[path])
    e.inject_random()
    res = e.step(200)
    assert res.converged == ro.converged and res.rounds == ro.rounds
    assert res.stats == ro.stats
    assert np.array_equal(res.infected, ro.infected)
    assert np.array_equal(e.read_shard(), full)
    e.close()
