"""Generates tests/golden/cfg4_oracle.json: configs[3] at full size (2^27 nodes, push-pull fanout 2,
64 rumors at their Philox origins, seed 0x5EED0004, to convergence) on the OpenMP C oracle
(oracle/gossip_oracle.c, the restatement of main.go:65-89 as rounds).

Stored: every round's stats (full, messages, state hash), the per-rumor infected counts, the
final state hash and the SHA-256 of the final state words ([N] uint64, little-endian).  Two
readers: the GPU tests (tests/test_gpu_cfg4_full.py, which also re-run the oracle live) and
bench.py, whose multi-GPU line checks its own run against this file ("verified"), so a sharded
run over RCCL that disseminated wrongly cannot report a rate.

    make -C oracle && python tests/golden/make_cfg4_golden.py   # ~2 min on 8 threads, ~3 GiB RAM
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

CFG4 = (1 << 27, 64, "pushpull", 2, 0x5EED0004)  # N, R, mode, fanout, seed
SAMPLE = (0, 1, 12345, (1 << 26) + 7, (1 << 27) - 1)


def state_digest(words: np.ndarray) -> str:
    return hashlib.sha256(memoryview(np.ascontiguousarray(words, dtype="<u8")).cast("B")).hexdigest()


def main():
    N, R, mode, k, seed = CFG4
    threads = int(os.environ.get("THREADS", os.cpu_count() or 1))
    o = op.OracleEngine(N, R, mode, k, seed, flags=1, threads=threads)
    o.inject_random()
    t0 = time.time()
    r = o.step(64)
    print(f"{r.rounds} rounds, {time.time() - t0:.0f} s, converged {r.converged}", flush=True)
    words = o.read_shard()[0]
    out = {"config": {"N": N, "R": R, "mode": mode, "fanout": k, "seed": hex(seed), "flags": 1,
                      "writes": "inject_random"},
           "generator": "tests/golden/make_cfg4_golden.py (oracle/gossip_oracle.c, OpenMP)",
           "rounds": r.rounds, "stats": r.stats, "infected": [[int(x) for x in row] for row in r.infected],
           "final_state_hash": int(o.state_hash()), "state_sha256": state_digest(words),
           "sample_words": {str(n): int(words[n]) for n in SAMPLE}}
    o.close()
    with open(os.path.join(HERE, "cfg4_oracle.json"), "w") as f:
        json.dump(out, f)
    print("wrote cfg4_oracle.json:", r.rounds, "rounds", out["state_sha256"])


if __name__ == "__main__":
    main()
