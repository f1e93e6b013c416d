"""Generates tests/golden/cfg5_oracle.json: configs[4] at full size (2^26 nodes, K = 16, fanout 1,
churn 1 % / 10 %, seed 0x5EED0005, one random write, to convergence) on the OpenMP C oracle
(oracle/gossip_oracle.c, the restatement of main.go:65-89 with each exchange one request/reply).

Stored: every round's stats (alive, full, messages, state hash), per-component counts, and the
SHA-256 of the final rows ([N][K] uint32, little-endian) with a few sampled rows.  The GPU tests
(tests/test_gpu_ae_sharded.py) compare the HIP engines with this file instead of re-running the
oracle on the GPU box, where it takes ~200 s of the suite (GOSSIP_CFG5_LIVE=1 re-runs it there).

    make -C oracle && python tests/golden/make_cfg5_golden.py   # ~10 min on 8 threads, ~10 GiB RAM
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))
import oracle_py as op  # noqa: E402
from gossip_hip.engine import churn_threshold as ct  # noqa: E402

CFG5 = (1 << 26, 16, 1, 0x5EED0005, 0.01, 0.1)  # N, K, fanout, seed, fail, recover
SAMPLE = (0, 1, 12345, (1 << 25) + 7, (1 << 26) - 1)


def rows_digest(rows: np.ndarray) -> str:
    return hashlib.sha256(memoryview(np.ascontiguousarray(rows, dtype="<u4")).cast("B")).hexdigest()


def main():
    N, K, k, seed, fail, rec = CFG5
    threads = int(os.environ.get("THREADS", os.cpu_count() or 1))
    o = op.OracleEngine(N, K, "antientropy", k, seed, flags=1, churn_fail=ct(fail), churn_recover=ct(rec),
                        threads=threads)
    o.inject_random()
    t0 = time.time()
    stats, inf = [], []
    while len(stats) < 400:
        r = o.step(10)
        stats += r.stats
        inf += [[int(x) for x in row] for row in r.infected]
        print(f"{len(stats)} rounds, {time.time() - t0:.0f} s", flush=True)
        if r.converged:
            break
    rows = o.read_rows()
    out = {"config": {"N": N, "K": K, "fanout": k, "seed": hex(seed), "churn_fail": fail, "churn_recover": rec,
                      "flags": 1, "writes": "inject_random"},
           "generator": "tests/golden/make_cfg5_golden.py (oracle/gossip_oracle.c, OpenMP)",
           "rounds": len(stats), "stats": stats, "infected": inf,
           "rows_sha256": rows_digest(rows), "sample_rows": {str(n): [int(x) for x in rows[n]] for n in SAMPLE}}
    with open(os.path.join(HERE, "cfg5_oracle.json"), "w") as f:
        json.dump(out, f)
    print("wrote cfg5_oracle.json:", len(stats), "rounds", out["rows_sha256"])


if __name__ == "__main__":
    main()
