#!/usr/bin/env python3
"""bench.py — gossip node-updates/sec on MI355X (BASELINE.json metric).

A step is one full dissemination run of the hot path: reset, inject the 64
rumors at their Philox origins, then push-pull rounds (fanout 2) until every
node holds every rumor.  node-updates = nodes x rounds.  The workload is the
north-star sweep, configs[3]: 2^27 nodes, push-pull k=2, R=64, seed
0x5EED0004, at every GPU count (1/2/4/8 GPUs, strong
scaling; N > 1 shards the node ids).  At one GPU the configs[2]
workload (2^24 nodes, seed 0x5EED0003) is timed beside it as `secondary`, and
configs[4] (anti-entropy with churn, 2^26 nodes x 16 versions) as `antientropy`.
State is resident in HBM; nothing crosses PCIe in the timed region except the
per-round 8-byte-per-rumor stats readback.

Single GPU:  python bench.py [--steps K --warmup W]
N GPUs:      python -m torch.distributed.run --nproc-per-node N bench.py --gpus N
Weak scaling instead (fixed nodes per GPU): --nodes-per-gpu M
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

NODES_TOTAL = 1 << 27      # configs[3], the north-star sweep (all GPU counts)
SEED_TOTAL = 0x5EED0004
NODES_SECONDARY = 1 << 24  # configs[2], one GPU
SEED_SECONDARY = 0x5EED0003
RUMORS = 64
FANOUT = 2
MODE = "pushpull"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ENGINE_PARAMS = {}  # gossip_set_param knobs of every engine the bench makes (--place-tries)
# configs[3] on the OpenMP C oracle (tests/golden/make_cfg4_golden.py): every run of that workload
# is checked against it, at every GPU count, before and after the timed steps
FIXTURE = os.path.join(ROOT, "tests", "golden", "cfg4_oracle.json")
STAT_KEYS = ("round", "converged", "full_nodes", "alive_nodes", "messages")


def alg_bytes_per_node_round(mode: str, k: int, words: int) -> int:
    """PULL 8W(2+k), PUSH 8W(2+2k), PUSH-PULL 8W(2+3k)."""
    return {"pull": 8 * words * (2 + k), "push": 8 * words * (2 + 2 * k),
            "pushpull": 8 * words * (2 + 3 * k)}[mode]


def load_pmc(workload: str):
    """PMC HBM traffic per dense round (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md §HBM), summed over
    the dense round's kernels, from the committed passes (tools/pmc_dense.py -> profiles/pmc_dense_*.json)."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_dense_*.json"))):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload:
            return d.get("hbm_bytes_per_dense_round"), os.path.relpath(path, ROOT)
    return None, None


def _omp_run(n_nodes: int, seed: int, threads: int, budget_s: float):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as op
    o = op.OracleEngine(n_nodes, RUMORS, MODE, FANOUT, seed, threads=threads)
    o.inject_random()
    rounds, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        res = o.step(1, with_infected=False)
        rounds += res.rounds
        if res.converged:
            break
    dt = time.perf_counter() - t0
    o.close()
    return n_nodes * rounds / dt, rounds, dt


def load_fixture(n_total: int, seed: int):
    """The oracle's run of this exact workload, or None (no fixture covers it)."""
    try:
        with open(FIXTURE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    c = d["config"]
    same = (c["N"], int(c["seed"], 16), c["R"], c["fanout"], c["mode"]) == (n_total, seed, RUMORS, FANOUT, MODE)
    return d if same else None


def global_state_hash(eng, world: int, backend: str) -> int:
    """DESIGN.md §2.5's state hash of the whole state: each shard hashes its own nodes (global ids)
    and the parts add up mod 2^64 (summed as four 16-bit limbs, so no collective overflows)."""
    h = eng.state_hash()
    if world == 1:
        return h
    limbs = torch.tensor([(h >> (16 * i)) & 0xFFFF for i in range(4)], dtype=torch.int64,
                         device="cuda" if backend == "nccl" else "cpu")
    dist.all_reduce(limbs, op=dist.ReduceOp.SUM)
    return sum(int(x) << (16 * i) for i, x in enumerate(limbs.tolist())) & ((1 << 64) - 1)


def check_run(stats: list, final_hash: int, fx: dict):
    """None when a step equals the oracle's run (per-round stats, final state hash), else what differs.
    The stats are global (all-reduced) and the hash is all-reduced, so every rank gets the same answer."""
    if len(stats) != fx["rounds"]:
        return f"{len(stats)} rounds, oracle {fx['rounds']}"
    for got, want in zip(stats, fx["stats"]):
        for key in STAT_KEYS:
            if int(got[key]) != int(want[key]):
                return f"round {want['round']}: {key} {int(got[key])}, oracle {int(want[key])}"
    if final_hash != fx["final_state_hash"]:
        return f"final state hash {final_hash:#x}, oracle {fx['final_state_hash']:#x}"
    return None


def cpu_baseline(n_nodes: int, seed: int, budget_s: float = 8.0):
    """The oracle (C restatement of the same rounds, `kind: port`; the reference itself is Go and not
    buildable here) on the host, same workload, bounded samples (whole rounds from the start of the run,
    about `budget_s` each): OpenMP on every CPU this process may run on, the job's host-core share
    (OMP_NUM_THREADS, 16 on the GPU box) and one thread.  The headline `value` / `cores` is the fastest
    of them (the oracle's random 8-B accesses share one memory system, so more threads can be slower:
    the baseline is not understated by a thread count that does not pay); all three are listed."""
    nproc = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = nproc
    share = max(1, min(avail, int(os.environ.get("OMP_NUM_THREADS", avail))))
    runs = {}
    v, rounds, dt = _omp_run(n_nodes, seed, avail, budget_s)
    runs["all_cpus"] = {"value": v, "cores": avail, "rounds": rounds, "seconds": dt,
                        "note": f"every affinity CPU (nproc {nproc})"}
    if share != avail:
        vs, rs, ds = _omp_run(n_nodes, seed, share, budget_s)
        runs["host_share"] = {"value": vs, "cores": share, "rounds": rs, "seconds": ds,
                              "note": "OMP_NUM_THREADS: this job's share of the host"}
    v1, rounds1, dt1 = _omp_run(n_nodes, seed, 1, budget_s)
    runs["single_thread"] = {"value": v1, "cores": 1, "rounds": rounds1, "seconds": dt1}
    best = max(runs, key=lambda k: runs[k]["value"])
    b = runs[best]
    counts = ", ".join(f"{r['cores']} threads" for r in runs.values())
    out = {"value": b["value"], "unit": "node-updates/s", "cores": b["cores"], "kind": "port",
           "nproc": nproc, "affinity_cpus": avail, "best_of": best,
           "sample": f"oracle/gossip_oracle.c, first {b['rounds']} rounds ({b['seconds']:.1f} s) of the same "
                     f"{n_nodes}-node push-pull k=2 R=64 run on {b['cores']} OpenMP threads (the fastest of "
                     f"{counts})"}
    out.update(runs)
    return out


def dense_only(n_nodes: int, seed: int, device: int, steps: int = 2):
    """Every round on the binned (dense) pipeline, same workload: the per-round cost the sparse
    frontier rounds avoid, reported beside the headline so that saving never hides in `frac`."""
    from gossip_hip import FLAG_DENSE, FLAG_TIMING, Engine
    # ahead 1: no round enqueued past convergence inside the timed region
    e = Engine(n_nodes, RUMORS, MODE, FANOUT, seed, flags=FLAG_TIMING | FLAG_DENSE, device=device,
               params={**ENGINE_PARAMS, "ahead": 1})
    e.reset(); e.inject_random(); e.step(64, with_infected=False)
    e.reset_timing()
    for _ in range(steps):
        e.reset(); e.inject_random(); e.step(64, with_infected=False)
    ms, n = e.kernel_time(3)
    e.close()
    us = ms * 1e3 / max(n, 1)
    bpn = alg_bytes_per_node_round(MODE, FANOUT, 1)
    return {"avg_round_us": us, "achieved_GBps": bpn * n_nodes / us / 1e3,
            "frac": bpn * n_nodes / us / 1e3 / HBM_PEAK_GBS, "rounds_timed": n,
            "note": "GOSSIP_FLAG_DENSE: every round of the step on the dense pipeline (also the nearly empty / "
                    "nearly full ones), same workload"}


def workload_name(nodes: int, world: int, per_gpu: bool) -> str:
    lg = int(np.log2(nodes))
    if per_gpu:
        return f"pushpull k=2 R=64, 2^{lg} nodes/GPU x {world}"
    return f"pushpull k=2 R=64, 2^{lg} nodes over {world} GPU" + ("s" if world > 1 else "")


def single_gpu_roofline(eng, nodes: int, workload: str) -> dict:
    """The dominant kernel group = the dense round (every kernel of one dense round), hipEvents around
    each dense round on the engine's stream inside the timed steps (engine timer 3)."""
    bpn = alg_bytes_per_node_round(MODE, FANOUT, 1)
    alg_round = bpn * nodes  # algorithmic bytes of one round
    dense_ms, dense_n = eng.kernel_time(3)
    sparse_ms, sparse_n = eng.kernel_time(4)
    step_ms, step_rounds = eng.kernel_time(0)
    dense_s = dense_ms / 1e3 / max(dense_n, 1)
    achieved = alg_round / dense_s / 1e9
    step_round_s = step_ms / 1e3 / max(step_rounds, 1)
    rl = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
          "frac": achieved / HBM_PEAK_GBS, "traffic": None,
          "bytes_per_node_round": bpn, "alg_bytes_per_launch": alg_round,
          "avg_launch_us": dense_s * 1e6, "rounds_timed": dense_n,
          "kernel": ("dense round = every kernel of one dense round (bin_emit, transpose, serve, apply; one "
                     "launch each), hipEvents around each dense round of the timed steps; achieved = 64 B x "
                     "nodes / average dense-round time (SURVEY.md §8(d))")}
    traffic, src = load_pmc(workload)
    if traffic:
        rl["traffic"] = traffic
        rl["traffic_ratio"] = traffic / alg_round
        rl["traffic_GBps"] = traffic / dense_s / 1e9
        rl["traffic_source"] = src
    rl["step_frac"] = {"achieved": alg_round / step_round_s / 1e9,
                       "frac": alg_round / step_round_s / 1e9 / HBM_PEAK_GBS,
                       "avg_round_us": step_round_s * 1e6, "rounds": step_rounds,
                       "note": "whole step (sparse rounds at the dense byte count, gaps included)"}
    rl["sparse_rounds"] = {"avg_round_us": sparse_ms * 1e3 / max(sparse_n, 1), "rounds_timed": sparse_n}
    return rl


def plan_model(eng, steps: int) -> dict:
    """N > 1: the planner's own price of the timed steps (gossip_plan_model) beside
    the measured line: its plan (one letter per round), the modelled per-rank wall per step (device
    time from the rates measured on one GPU + link bytes over link_gbps per xGMI link) and its link
    part.  A real N-GPU line then shows at once whether the link rate the model assumes holds."""
    ms, link, n, plan = eng.plan_model()
    return {"plan": plan, "model_wall_ms": ms / max(steps, 1), "model_link_ms": link / max(steps, 1),
            "model_device_ms": (ms - link) / max(steps, 1), "rounds_modelled": int(n // max(steps, 1)),
            "link_gbps": ENGINE_PARAMS.get("link_gbps", 76.0),
            "what": "per step and rank: S sparse, X exchange, C class-coded, D state all-gather dense rounds, "
                    "R / Q replicated after the state / class-coded all-gather, r replicated on the whole image "
                    "(no collective)"}


def sharded_roofline(eng, driver: str, trace, alg_round: int, world: int, backend: str, steps: int = 1) -> dict:
    """N > 1: the dense round's fraction of the HBM roofline on WHOLE-round time per rank (plan,
    collectives over the links, kernels, host reads), from hipEvents around each round of the
    timed steps on the stream the collectives are ordered on (torch driver: torch.cuda.Event
    pairs in gossip_hip.sharded.sharded_run; engine driver: gossip_round_wall).  The device work
    alone (engine timer 0, collectives excluded) is reported beside it, with the link bytes this
    rank sent per round (the collectives' sizes)."""
    dense_ms = dense_n = dense_link = sparse_ms = sparse_n = sparse_link = 0.0
    if driver == "engine":
        dense_ms, dense_n, dense_link = eng.round_wall(0)
        sparse_ms, sparse_n, sparse_link = eng.round_wall(1)
    elif trace:
        for r in trace:
            ms = r["events"][0].elapsed_time(r["events"][1]) if "events" in r else 0.0
            if r["kind"] == 1:
                sparse_ms, sparse_n, sparse_link = sparse_ms + ms, sparse_n + 1, sparse_link + r["link_bytes"]
            else:
                dense_ms, dense_n, dense_link = dense_ms + ms, dense_n + 1, dense_link + r["link_bytes"]
    round_s = dense_ms / 1e3 / max(dense_n, 1)
    dev_ms, dev_n = eng.kernel_time(0)
    dev_s = dev_ms / 1e3 / max(dev_n, 1)
    achieved = alg_round / round_s / 1e9 if round_s > 0 else 0.0
    dev_achieved = alg_round / dev_s / 1e9 if dev_s > 0 else 0.0
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None, "bytes_per_node_round": alg_round // max(eng.hi - eng.lo, 1),
            "alg_bytes_per_launch": alg_round, "avg_launch_us": round_s * 1e6,
            "round_wall_us": round_s * 1e6, "dense_rounds_timed": int(dense_n),
            "link_bytes_per_round": dense_link / max(dense_n, 1),
            "sparse_round_wall_us": sparse_ms * 1e3 / max(sparse_n, 1), "sparse_rounds_timed": int(sparse_n),
            "link_bytes_per_sparse_round": sparse_link / max(sparse_n, 1),
            "device_only": {"avg_round_us": dev_s * 1e6, "rounds": int(dev_n), "frac": dev_achieved / HBM_PEAK_GBS,
                            "what": "engine timer 0: the hot kernels' device time per round, collectives excluded"},
            "plan_model": plan_model(eng, steps),
            "kernel": ("sharded dense rounds, each timed whole per rank: plan, collectives (state all-gather, "
                       "class-coded all-gather or exchange all-to-alls), kernels and host reads, from hipEvents on "
                       "the stream the collectives are ordered on; alg bytes = 64 B x own nodes"
                       + (" (gloo rehearsal: collectives staged through the host, not a link measurement)"
                          if backend == "gloo" else ""))}


def secondary_run(device: int, steps: int, warmup: int) -> dict:
    """configs[2] on the same GPU (2^24 nodes: the state fits the 256 MiB Infinity Cache), same step."""
    from gossip_hip import FLAG_TIMING, Engine
    n = NODES_SECONDARY
    e = Engine(n, RUMORS, MODE, FANOUT, SEED_SECONDARY, flags=FLAG_TIMING, device=device, params=dict(ENGINE_PARAMS))

    def one():
        e.reset(); e.inject_random()
        return e.step(64, with_infected=False)
    for _ in range(warmup):
        one()
    e.reset_timing()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rounds = 0
    for _ in range(steps):
        res = one()
        assert res.converged
        rounds += res.rounds
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    wl = workload_name(n, 1, False)
    rl = single_gpu_roofline(e, n, wl)
    e.close()
    return {"workload": wl, "nodes": n, "seed": hex(SEED_SECONDARY), "value": n * rounds / dt,
            "ms_per_step": dt * 1e3 / steps, "rounds_to_converge": rounds // steps,
            "roofline_frac": rl["frac"], "avg_dense_round_us": rl["avg_launch_us"],
            "traffic": rl["traffic"], "step_frac": rl["step_frac"]["frac"],
            "sparse_avg_round_us": rl["sparse_rounds"]["avg_round_us"]}


def antientropy_run(device: int, steps: int, warmup: int) -> dict:
    """configs[4] on the same GPU: 2^26 nodes x K = 16 u32 versions, k = 1, churn 1 % / 10 %,
    seed 0x5EED0005, a random write, rounds to convergence.  No per-round state
    hash (flag 1: the parity tests' check; the reference keeps none).  Dense rounds are priced at
    SURVEY.md §8(d)'s 4K(2 + 2k) = 256 B per node-round."""
    from gossip_hip import FLAG_TIMING, Engine, loss_threshold
    n, K, k, seed = 1 << 26, 16, 1, 0x5EED0005
    e = Engine(n, K, "antientropy", k, seed, flags=FLAG_TIMING, device=device, params=dict(ENGINE_PARAMS),
               churn_fail=loss_threshold(0.01), churn_recover=loss_threshold(0.1))

    def one():
        e.reset(); e.inject_random()
        return e.step(400, with_infected=False)
    for _ in range(warmup):
        one()
    # the per-round split from timed runs; the time to converge from as many untimed runs on the
    # same engine (param timing 0: no hipEvent between rounds, ~0.9 ms per run)
    e.reset_timing()
    for _ in range(steps):
        assert one().converged
    dense_ms, dense_n = e.kernel_time(0)
    sparse_ms, sparse_n = e.kernel_time(2)
    e.set_param("timing", 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rounds = 0
    for _ in range(steps):
        res = one()
        assert res.converged
        rounds += res.rounds
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    e.close()
    dense_us = dense_ms * 1e3 / max(dense_n, 1)
    achieved = 4 * K * (2 + 2 * k) * n / (dense_us * 1e-6) / 1e9
    return {"workload": "antientropy K=16 k=1 churn 1%/10%, 2^26 nodes over 1 GPU (configs[4])", "nodes": n,
            "seed": hex(seed), "value": n * rounds / dt, "unit": "node-updates/s",
            "ms_to_converge": dt * 1e3 / steps, "rounds_to_converge": rounds // steps,
            "dense_rounds": dense_n // steps, "avg_dense_round_us": dense_us,
            "dense_round_roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": achieved / HBM_PEAK_GBS, "bytes_per_node_round": 4 * K * (2 + 2 * k)},
            "sparse_rounds": sparse_n // steps, "avg_sparse_round_us": sparse_ms * 1e3 / max(sparse_n, 1),
            "state_hash": False}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=NODES_TOTAL, help="total nodes (strong scaling; default 2^27)")
    ap.add_argument("--nodes-per-gpu", type=int, default=0, help="weak scaling: this many nodes per GPU")
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dense-only", action="store_true", help="skip the all-dense comparison run (profiling)")
    ap.add_argument("--no-secondary", action="store_true", help="skip the configs[2] line (profiling)")
    ap.add_argument("--no-antientropy", action="store_true", help="skip the configs[4] line (profiling)")
    ap.add_argument("--place-tries", type=int, default=0,
                    help="engine param place_tries (0: the engine's default; 1: no placement trial rounds, "
                         "for PMC passes that should count only the workload's rounds)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="collectives for N > 1: nccl (= RCCL, the measured path) or gloo (a rehearsal of the "
                         "multi-rank code on a box with fewer GPUs than ranks: ranks share devices; --driver torch)")
    ap.add_argument("--driver", default=None, choices=("engine", "torch"),
                    help="N > 1: torch (default) = gossip_hip.sharded drives the rounds over torch.distributed "
                         "(RCCL); engine = the library runs every sharded round over its own RCCL communicator "
                         "(gossip_comm_init_rank + gossip_step, DESIGN.md §5.5; not yet run on distinct GPUs, so "
                         "opt-in: a run that differs from the oracle fixture falls back to torch)")
    args = ap.parse_args()
    if args.place_tries:
        ENGINE_PARAMS["place_tries"] = args.place_tries

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    if args.backend == "gloo":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world > 1 and args.backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    elif world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from gossip_hip import FLAG_TIMING, Engine
    from gossip_hip.sharded import sharded_run

    per_gpu = args.nodes_per_gpu > 0
    n_total = args.nodes_per_gpu * world if per_gpu else args.nodes
    if args.seed is not None:
        seed = args.seed
    else:
        seed = SEED_TOTAL if n_total >= NODES_TOTAL or world > 1 else SEED_SECONDARY
    mem_free0 = torch.cuda.mem_get_info()[0] if world == 1 else None
    t_create = time.perf_counter()
    eng = Engine(n_total, RUMORS, MODE, FANOUT, seed, flags=FLAG_TIMING, device=local,
                 shard_rank=rank, shard_count=world, params=dict(ENGINE_PARAMS))
    create_ms = (time.perf_counter() - t_create) * 1e3
    mem_free1 = torch.cuda.mem_get_info()[0] if world == 1 else None
    driver = (args.driver or "torch") if world > 1 else "engine"
    driver_note = None
    if world > 1 and driver == "engine" and args.backend == "gloo":
        driver, driver_note = "torch", "gloo rehearsal: ranks share devices, which RCCL refuses"
    if world > 1 and driver == "engine":
        from gossip_hip.sharded import init_engine_comm
        why = init_engine_comm(eng)  # collective: every rank gets the same answer
        if why:  # report it in the line, and measure the torch-driven rounds instead
            driver, driver_note = "torch", f"engine RCCL init failed: {why}"
            print(f"warning: {driver_note}", file=sys.stderr)

    def use_torch_driver():
        eng.set_stream(torch.cuda.current_stream().cuda_stream)

    if world > 1 and driver == "torch":
        use_torch_driver()

    trace = None  # torch driver, timed steps: per round {"kind", "link_bytes", "events"}

    def one_step():
        eng.reset()
        eng.inject_random()
        if driver == "engine":  # one GPU, or every rank in gossip_step over the engine's RCCL comm
            return eng.step(64, with_infected=False).stats
        return sharded_run(eng, 64, trace=trace)

    fx = load_fixture(n_total, seed)

    def verify(stats):
        if fx is None:
            return "no oracle fixture for this workload"
        return check_run(stats, global_state_hash(eng, world, args.backend), fx)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    warm_check = None
    engine_driver_verified = None  # N > 1, --driver engine: did the library-driven run match the fixture?
    first_step = None  # one GPU: wall time and least free device memory of the first step (its placement trials)
    for i in range(args.warmup):
        if i == 0 and world == 1:
            # (no memory sampling here: a thread polling hipMemGetInfo during the trials made this
            # step 3.9 s instead of ~0.24 s; tools/place_seq.py measures the peak separately)
            t_first = time.perf_counter()
            st = one_step()
            first_step = ((time.perf_counter() - t_first) * 1e3, mem_free1 - torch.cuda.mem_get_info()[0])
        else:
            st = one_step()
        if i == 0 and fx is not None:  # before the timed steps: a wrong result is caught, not timed
            warm_check = verify(st)
            if world > 1 and driver == "engine":
                engine_driver_verified = warm_check is None
            if warm_check and world > 1 and driver == "engine":
                driver_note = (f"the engine-driven run differed from the oracle fixture ({warm_check}): the "
                               "rounds are driven over torch.distributed instead")
                print(f"warning: {driver_note}", file=sys.stderr)
                if args.driver == "engine":  # asked for explicitly: a wrong library result fails the run
                    print("error: --driver engine gave a wrong result", file=sys.stderr)
                    if world > 1:
                        dist.destroy_process_group()
                    sys.exit(3)
                driver = "torch"
                use_torch_driver()
    placement = eng.kernel_time(5)  # the record slab's placement trial rounds, in warm-up
    eng.reset_timing()
    if world > 1 and driver == "torch":
        trace = []
    barrier()
    t0 = time.perf_counter()
    rounds, last = [], None
    for _ in range(args.steps):
        last = one_step()
        assert last[-1]["converged"], "run did not converge within 64 rounds"
        rounds.append(len(last))
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device="cuda" if args.backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # after the timed region: the last timed step against the oracle's run of the same workload
    final_check = verify(last) if last is not None else "no timed step"
    verified = None if fx is None or last is None else final_check is None

    total_rounds = sum(rounds)
    value = n_total * total_rounds / dt
    nown = eng.hi - eng.lo
    bpn = alg_bytes_per_node_round(MODE, FANOUT, 1)
    workload = workload_name(args.nodes_per_gpu if per_gpu else n_total, world, per_gpu)
    if world == 1:
        rl = single_gpu_roofline(eng, n_total, workload)
        rl["placement_trials"] = {"launches": placement[1], "ms": placement[0],
                                  "note": "serve launches timed on fresh allocations of the record slab (one emit "
                                          "each, not counted) before the first round (param place_tries, DESIGN.md "
                                          "\u00a73.7), in the warm-up: not in the timed steps"}
        if first_step is not None:
            rl["engine_setup"] = {
                "create_ms": round(create_ms, 1), "device_bytes_after_create": int(mem_free0 - mem_free1),
                "first_step_ms": round(first_step[0], 1), "timed_step_ms": round(dt / max(args.steps, 1) * 1e3, 2),
                "extra_device_bytes_after_first_step": int(first_step[1]),
                "note": "gossip_create wall time and the device memory it took; the first step's wall time (it runs "
                        "the placement trials, which hold at most two candidate record slabs beside the kept one: "
                        "DESIGN.md §3.7, peak measured by tools/place_seq.py) and what it left allocated"}
    else:
        rl = sharded_roofline(eng, driver, trace, bpn * nown, world, args.backend, args.steps)
    eng.close()

    if rank == 0:
        out = {
            "metric": "gossip node-updates/sec (nodes x rounds)",
            "value": value,
            "unit": "node-updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak" if per_gpu else "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (64 rumors injected at Philox tag-2 origins)",
            "config": {"workload": workload, "nodes": n_total, "nodes_per_gpu": nown, "rumors": RUMORS,
                       "fanout": FANOUT, "mode": MODE, "seed": hex(seed), "rounds_to_converge": rounds[0],
                       "parallelism": f"shard{world}" if world > 1 else "single",
                       **({"driver": driver} if world > 1 else {}),
                       **({"driver_note": driver_note} if driver_note else {})},
            "verified": verified,
            **({"engine_driver_verified": engine_driver_verified} if engine_driver_verified is not None else {}),
            "verification": (f"per-round stats ({', '.join(STAT_KEYS)}) and the final state hash of the last "
                             f"timed step{' (all ranks, hash summed over the shards)' if world > 1 else ''} equal "
                             f"the OpenMP oracle's run of the same workload ({os.path.relpath(FIXTURE, ROOT)})"
                             if verified else final_check),
            **({"backend": "gloo (rehearsal: not a measurement)"} if world > 1 and args.backend == "gloo" else {}),
            "roofline": rl,
        }
        if world == 1 and not args.no_dense_only:
            rl["dense_only"] = dense_only(n_total, seed, local)
        if world == 1 and not args.no_secondary and n_total != NODES_SECONDARY:
            out["secondary"] = secondary_run(local, max(args.steps, 5), max(args.warmup, 2))
        if world == 1 and not args.no_antientropy and not per_gpu and n_total == NODES_TOTAL:
            out["antientropy"] = antientropy_run(local, 3, 1)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(n_total, seed)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
