"""GPU, two processes on one device: the sharded round protocol through real
process boundaries (gloo collectives staged through host memory) with HIP
shard engines equals a single-engine run bit for bit.  On a multi-GPU node
the same code path uses RCCL (backend "nccl") instead."""
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


def _worker(rank, world, port, case, q):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "gossip-protocol_amd")]
    import torch
    import torch.distributed as dist
    from gossip_hip import Engine
    from gossip_hip.sharded import sharded_run
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mode, k, R, N, seed = case
    e = Engine(N, R, mode, k, seed, flags=1, device=0, shard_rank=rank, shard_count=world)
    e.inject_random()
    stats = sharded_run(e, 100)
    q.put((rank, e.lo, e.hi, stats, e.read_shard()))
    dist.destroy_process_group()


@pytest.mark.parametrize("case", [("pushpull", 2, 64, 1 << 20, 0x5EED0004), ("push", 3, 1, 300001, 7)],
                         ids=["pushpull-1M", "push-ragged"])
def test_two_processes_equal_one_engine(case):
    from gossip_hip import Engine
    mode, k, R, N, seed = case
    ref = Engine(N, R, mode, k, seed, flags=1, device=0)
    ref.inject_random()
    want = ref.step(100)
    full = ref.read_shard()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=180) for _ in range(2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, lo, hi, stats, shard in got:
        assert stats == want.stats
        assert np.array_equal(shard, full[:, lo:hi])
