"""CPU: bench.py's self-check.  Every bench run of configs[3] compares its per-round
stats and final state hash with the OpenMP oracle's run of the same workload
(tests/golden/cfg4_oracle.json), before and after the timed steps and at every GPU count, so a
multi-GPU line cannot report a rate for a wrong dissemination."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_fixture_matches_the_bench_workload_only():
    fx = bench.load_fixture(bench.NODES_TOTAL, bench.SEED_TOTAL)
    assert fx is not None and fx["rounds"] == 15
    assert bench.load_fixture(bench.NODES_SECONDARY, bench.SEED_SECONDARY) is None
    assert bench.load_fixture(bench.NODES_TOTAL, bench.SEED_TOTAL + 1) is None


def test_check_run_accepts_the_oracle_run_and_names_a_difference():
    fx = bench.load_fixture(bench.NODES_TOTAL, bench.SEED_TOTAL)
    stats = copy.deepcopy(fx["stats"])
    for s in stats:
        s["state_hash"] = 0  # the bench's engines run without the per-round hash
    assert bench.check_run(stats, fx["final_state_hash"], fx) is None
    bad = copy.deepcopy(stats)
    bad[9]["full_nodes"] += 1
    assert "round 9: full_nodes" in bench.check_run(bad, fx["final_state_hash"], fx)
    assert "rounds" in bench.check_run(stats[:-1], fx["final_state_hash"], fx)
    assert "hash" in bench.check_run(stats, fx["final_state_hash"] ^ 1, fx)
