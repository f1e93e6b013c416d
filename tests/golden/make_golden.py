"""Generates tests/golden/golden.json from the independent numpy restatement
(oracle/numpy_ref.py).  TEST INFRASTRUCTURE: the reference (Go) has no tests,
fixtures or runnable toolchain here, so these vectors pin the C oracle and the
HIP engine to a second, separately written restatement of DESIGN.md §2.

Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))

import numpy_ref as nr  # noqa: E402
from gossip_hip.maelstrom import grid_topology, line_topology, total_topology, tree_topology  # noqa: E402

KAT = [  # Random123 kat_vectors for philox4x32_10 (also checked against rocRAND's ten_rounds)
    {"ctr": [0, 0, 0, 0], "key": [0, 0], "out": [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]},
    {"ctr": [0xffffffff] * 4, "key": [0xffffffff] * 2, "out": [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]},
    {"ctr": [0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], "key": [0xa4093822, 0x299f31d0],
     "out": [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]},
]

RANDOM_CASES = [
    # name, N, R, mode, k, seed, injection ("random" or [(node, rumor), ...])
    ("push_k3_r1", 4096, 1, "push", 3, 0x5EED0001, [(0, 0)]),
    ("push_k1_r1", 2048, 1, "push", 1, 0x5EED0001, [(0, 0)]),
    ("pull_k2_r1", 4096, 1, "pull", 2, 0x5EED0002, [(7, 0)]),
    ("pushpull_k2_r64", 4096, 64, "pushpull", 2, 0x5EED0003, "random"),
    ("pushpull_k2_r1_small", 2, 1, "pushpull", 2, 1, [(1, 0)]),
    ("pushpull_k3_r130", 1500, 130, "pushpull", 3, 0xABCDEF0123456789, "random"),
    ("push_k5_r70", 777, 70, "push", 5, 42, "random"),
    ("pull_k6_r64_ragged", 1023, 64, "pull", 6, 0xFFFFFFFF00000001, "random"),
]


def adj(topo, n):
    return [[int(v[1:]) for v in topo[f"n{i}"]] for i in range(n)]


FLOOD_CASES = [
    ("grid25_n0", 25, 1, adj(grid_topology(25), 25), [(0, 0)]),
    ("grid25_all_origins", 25, 25, adj(grid_topology(25), 25), [(i, i) for i in range(25)]),
    ("grid5_n0", 5, 1, adj(grid_topology(5), 5), [(0, 0)]),
    ("line16_mid", 16, 1, adj(line_topology(16), 16), [(7, 0)]),
    ("tree3_40", 40, 2, adj(tree_topology(40, 3), 40), [(0, 0), (39, 1)]),
    ("total8", 8, 1, adj(total_topology(8), 8), [(3, 0)]),
    # directed, asymmetric, with a duplicate edge and a self loop; disconnected node 5
    ("directed_ring", 6, 2, [[1, 1], [2], [3, 0], [4], [0, 4], [5]], [(0, 0), (2, 1)]),
]


LOSS = lambda p: min(int(round(p * 2**32)), 2**32 - 1)  # noqa: E731  (gossip_hip.loss_threshold)

# random modes under faults and the stall mode (§2.9): name, N, R, mode, k, seed,
# injection, edge_loss, partitions, stall_rounds, max_rounds
RANDOM_FAULT_CASES = [
    ("pushpull_loss30", 2000, 8, "pushpull", 2, 9, "random", LOSS(0.3), 0, 0, 200),
    ("pushpull_stall3_loss10", 3000, 64, "pushpull", 2, 0x5EED0003, "random", LOSS(0.1), 0, 3, 200),
    ("push_stall2_parts2", 2001, 1, "push", 3, 7, [(0, 0), (1500, 0)], LOSS(0.05), 2, 2, 60),
    ("pull_stall1_loss2", 1500, 5, "pull", 2, 11, "random", LOSS(0.02), 0, 1, 200),
    ("pushpull_k6_stall4", 1000, 7, "pushpull", 6, 3, "random", LOSS(0.25), 2, 4, 80),
]

# FLOOD with faults: one walk per (node, value) down the node's row in the topology message's
# order, head-of-line blocked by a lost attempt, stuck for good after stall_rounds lost attempts on
# one neighbour (§2.9; main.go:72-87):
# name, N, R, adjacency, injection, edge_loss, partitions, stall_rounds, max_rounds
FLOOD_FAULT_CASES = [
    # node 0's first neighbour sits across the partition: the walk never gets past it, so 1 and 2
    # never hear from 0 (the same row in another order reaches them in round 0)
    ("hol_partition_blocked", 6, 1, [[3, 1, 2], [0], [0], [4], [5], []], [(0, 0)], 0, 2, 0, 12),
    ("hol_partition_blocked_stall1", 6, 1, [[3, 1, 2], [0], [0], [4], [5], []], [(0, 0)], 0, 2, 1, 12),
    ("hol_partition_order", 6, 1, [[1, 2, 3], [0], [0], [4], [5], []], [(0, 0)], 0, 2, 1, 12),
    ("grid25_loss30_stall1", 25, 3, adj(grid_topology(25), 25), [(0, 0), (24, 1), (12, 2)], LOSS(0.3), 0, 1, 80),
    ("grid25_loss30_retry", 25, 2, adj(grid_topology(25), 25), [(0, 0), (24, 1)], LOSS(0.3), 0, 0, 80),
    ("grid25_loss30_stall2", 25, 2, adj(grid_topology(25), 25), [(0, 0), (24, 1)], LOSS(0.3), 0, 2, 80),
    ("tree3_40_parts2_stall3", 40, 2, adj(tree_topology(40, 3), 40), [(0, 0), (39, 1)], LOSS(0.1), 2, 3, 60),
    ("directed_ring_loss50_stall1", 6, 2, [[1, 1], [2], [3, 0], [4], [0, 4], [5]], [(0, 0), (2, 1)],
     LOSS(0.5), 0, 1, 40),
    ("line16_parts4_retry", 16, 1, adj(line_topology(16), 16), [(7, 0)], 0, 4, 0, 30),
    ("grid25_70vals_loss20_stall3", 25, 70, adj(grid_topology(25), 25), [(i % 25, i) for i in range(70)],
     LOSS(0.2), 0, 3, 80),
]

AE_CASES = [
    # name, N, K, fanout, seed, fail, recover  (thresholds = probability * 2^32)
    ("ae_cfg5_small", 4096, 16, 1, 0x5EED0005, int(0.01 * 2**32), int(0.1 * 2**32)),
    ("ae_heavy_churn", 1000, 5, 2, 7, int(0.2 * 2**32), int(0.3 * 2**32)),
    ("ae_no_churn_k64", 513, 64, 1, 3, 0, 0),
]


def run_case(sim, inj, max_rounds=256):
    if inj == "random":
        sim.inject_random()
    else:
        for n, r in inj:
            sim.inject(n, r)
    rounds = sim.run(max_rounds)
    return [{k: (int(v) if not isinstance(v, list) else v) for k, v in st.items()} for st in rounds]


def main():
    out = {"philox_kat": KAT, "peers": [], "origins": [], "random": [], "flood": [], "antientropy": [],
           "random_faults": [], "flood_faults": []}
    for seed, N, t in [(0x5EED0001, 1 << 20, 0), (0x5EED0003, 1 << 24, 5), (7, 1000, 3), (0, 2, 0)]:
        nodes = sorted(set([i for i in range(16) if i < N] + [N - 1]))
        p = nr.peers(seed, N, t, 6, nodes=nodes)
        out["peers"].append({"seed": seed, "N": N, "t": t, "nodes": nodes,
                             "peers": [[int(x) for x in row] for row in p]})
    for seed, N, R in [(0x5EED0003, 1 << 24, 64), (1, 1000, 10)]:
        out["origins"].append({"seed": seed, "N": N, "R": R,
                               "origins": [int(x) for x in nr.origins(seed, N, R)]})
    for name, N, R, mode, k, seed, inj in RANDOM_CASES:
        sim = nr.Sim(N, R, mode, k, seed)
        rounds = run_case(sim, inj)
        out["random"].append({"name": name, "N": N, "R": R, "mode": mode, "k": k, "seed": seed,
                              "inject": inj, "rounds": rounds, "final_hash": nr.state_hash(sim.S)})
    for name, N, R, A, inj in FLOOD_CASES:
        sim = nr.Sim(N, R, "flood", topology=A)
        rounds = run_case(sim, inj)
        reads = {i: [r for r in range(R) if (int(sim.S[r // 64, i]) >> (r % 64)) & 1] for i in range(N)}
        out["flood"].append({"name": name, "N": N, "R": R, "adj": A, "inject": inj, "rounds": rounds,
                             "reads": reads})
    for name, N, R, mode, k, seed, inj, loss, parts, stall, mr in RANDOM_FAULT_CASES:
        sim = nr.Sim(N, R, mode, k, seed, edge_loss=loss, partitions=parts, stall_rounds=stall)
        rounds = run_case(sim, inj, mr)
        out["random_faults"].append({"name": name, "N": N, "R": R, "mode": mode, "k": k, "seed": seed,
                                     "inject": inj, "edge_loss": loss, "partitions": parts, "stall_rounds": stall,
                                     "max_rounds": mr, "rounds": rounds, "final_hash": nr.state_hash(sim.S),
                                     "stalled": int((sim.streak >= stall).sum()) if stall else 0})
    for name, N, R, A, inj, loss, parts, stall, mr in FLOOD_FAULT_CASES:
        sim = nr.Sim(N, R, "flood", topology=A, edge_loss=loss, partitions=parts, stall_rounds=stall)
        rounds = run_case(sim, inj, mr)
        reads = {i: [r for r in range(R) if (int(sim.S[r // 64, i]) >> (r % 64)) & 1] for i in range(N)}
        out["flood_faults"].append({"name": name, "N": N, "R": R, "adj": A, "inject": inj, "edge_loss": loss,
                                    "partitions": parts, "stall_rounds": stall, "max_rounds": mr,
                                    "rounds": rounds, "reads": reads})
    for name, N, K, k, seed, fail, rec in AE_CASES:
        sim = nr.AntiEntropySim(N, K, k, seed, fail, rec)
        sim.inject_random()
        sim.inject(N - 1, 0)  # a client write after the initial versions
        rounds = sim.run(300)
        out["antientropy"].append({"name": name, "N": N, "K": K, "k": k, "seed": seed, "fail": fail,
                                   "recover": rec, "rounds": rounds,
                                   "node0": [int(x) for x in sim.V[0]], "node0_alive": bool(sim.alive[0])})
    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
