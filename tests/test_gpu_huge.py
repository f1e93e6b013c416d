"""GPU, the one-shard dense rounds past 2^26 nodes with 32768-sender regions against the OpenMP oracle.

Past 4096 destination tiles (N > 2^26) with fanout <= 2 the dense emit bins 32768-sender regions
(binned.hip bin_emit_huge_kernel): the peers stay in registers, the records are written in two
passes over halves of the tiles, the run offsets are kept mod 2^16 with exact totals per region,
and the apply's reply walk takes its half of a region's records (a tile is half a region).  Every
path must equal the oracle bit for bit: per-round stats, per-rumor counts and the final state.
N = 2^26 + 4099: 4097 tiles, a ragged last region (4099 senders) and a ragged last tile.
Reference: (*NodeState).Gossip, main.go:65-89, as rounds.
"""
import os

import numpy as np
import pytest

import oracle_py as op
from gossip_hip import Engine

pytestmark = pytest.mark.gpu

N = (1 << 26) + 4099
THREADS = min(16, os.cpu_count() or 1)
ROUNDS = 40
# auto: as planned (sparse and dense rounds); dense: every round on the dense pipeline; dense_filter:
# every round dense with the edge filter (empty / full peers' one-way edges dropped in the emit)
PATHS = {"auto": {}, "dense": {"sparse_frac": -1.0},
         "dense_filter": {"sparse_frac": -1.0, "filter_frac": 0.3}}
CASES = {"pushpull-k2-R64": ("pushpull", 2, 64, 0x5EED0003, 0, 0),
         "push-k2-R5": ("push", 2, 5, 77, 0, 0),
         "pull-k1-R3": ("pull", 1, 3, 0x51, 0, 0),
         # edge loss: the emit's fault branch (FAULTS)
         "pushpull-k2-R7-loss": ("pushpull", 2, 7, 9, 1 << 30, 0)}


@pytest.fixture(scope="module")
def oracle_runs():
    cache = {}

    def get(case):
        if case not in cache:
            mode, k, r, seed, loss, parts = CASES[case]
            o = op.OracleEngine(N, r, mode, k, seed, flags=1, threads=THREADS, edge_loss=loss, partitions=parts)
            o.inject_random()
            res = o.step(ROUNDS)
            cache[case] = (res, o.read_shard())
            o.close()
        return cache[case]
    return get


@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("path", list(PATHS))
def test_huge_regions_equal_oracle(oracle_runs, case, path):
    mode, k, r, seed, loss, parts = CASES[case]
    ro, full = oracle_runs(case)
    e = Engine(N, r, mode, k, seed, flags=1, edge_loss=loss, partitions=parts, params=PATHS[path])
    e.inject_random()
    res = e.step(ROUNDS)
    assert res.converged == ro.converged and res.rounds == ro.rounds
    assert res.stats == ro.stats
    assert np.array_equal(res.infected, ro.infected)
    assert np.array_equal(e.read_shard(), full)
    e.close()
