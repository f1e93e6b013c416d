"""GPU, two processes: the sharded round protocol through real process
boundaries with HIP shard engines equals a single-engine run bit for bit.

  gloo — both ranks on device 0, collectives staged through host memory;
  gloo-dev — both ranks on device 0, the RCCL branch of gossip_hip.sharded forced
         (direct=True): gloo's device collectives on engine memory in place, the
         all-gathers async with work.wait(), the engines bound to torch's stream;
  nccl — RCCL collectives on engine memory, in place, with the engines bound to
         torch's current stream (gossip_hip.sharded._bind_stream).  Needs two
         devices (RCCL rejects two ranks on one GPU); skipped on a one-GPU box;
  engine — every round inside the library (gossip_comm_unique_id /
         gossip_comm_init_rank through gossip_hip.sharded.init_engine_comm, then
         gossip_step: the engine's own RCCL communicator), the
         path `bench.py --driver engine` measures.  Needs two devices likewise."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q, backend="gloo"):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "gossip-protocol_amd")]
    import torch
    import torch.distributed as dist
    from gossip_hip import Engine
    from gossip_hip.sharded import sharded_run
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    rccl = backend in ("nccl", "engine")
    dev = rank if rccl else 0
    torch.cuda.set_device(dev)
    direct = True if backend == "gloo-dev" else None
    if rccl:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", dev))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    mode, k, R, N, seed, params = case
    kw = _ae_kw(mode)
    e = Engine(N, R, mode, k, seed, flags=1, device=dev, shard_rank=rank, shard_count=world, params=params, **kw)
    e.inject_random()
    if backend == "engine":
        from gossip_hip.sharded import init_engine_comm
        why = init_engine_comm(e)
        assert why is None, why
        stats = e.step(400).stats
    else:
        stats = sharded_run(e, 400, direct=direct)
    q.put((rank, e.lo, e.hi, stats, _state(e)))
    dist.destroy_process_group()


def _ae_kw(mode):
    from gossip_hip.engine import churn_threshold as ct
    return dict(churn_fail=ct(0.01), churn_recover=ct(0.1)) if mode == "antientropy" else {}


def _state(e):
    return e.read_rows() if e.cfg.mode == 4 else e.read_shard()


CASES = [("pushpull", 2, 64, 1 << 20, 0x5EED0004, None),
         ("push", 3, 1, 300001, 7, None),
         ("pushpull", 2, 64, (1 << 20) + 77, 0x5EED0004, {"xd_shards": 2}),  # dense rounds as exchange rounds
         ("antientropy", 1, 16, 1 << 18, 0x5EED0005, None),
         # dense rounds replicated (kinds 5 / 6): all-gather once, then no collective
         ("pushpull", 2, 64, (1 << 20) + 3, 0x5EED0004, {"replicate": 1})]


@pytest.mark.parametrize("backend", ["gloo", "gloo-dev", "nccl", "engine"])
@pytest.mark.parametrize("case", CASES, ids=["pushpull-1M", "push-ragged", "pushpull-exchange", "antientropy",
                                           "pushpull-replicated"])
def test_two_processes_equal_one_engine(case, backend):
    import torch
    if backend in ("nccl", "engine") and torch.cuda.device_count() < 2:
        pytest.skip("RCCL needs one device per rank")
    from gossip_hip import Engine
    mode, k, R, N, seed, _ = case
    ref = Engine(N, R, mode, k, seed, flags=1, device=0, **_ae_kw(mode))
    ref.inject_random()
    want = ref.step(400)
    full = _state(ref)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, q, backend)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in range(2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, lo, hi, stats, shard in got:
        assert stats == want.stats
        assert np.array_equal(shard, full[lo:hi] if mode == "antientropy" else full[:, lo:hi])
