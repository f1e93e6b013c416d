"""Sharded rounds across ranks: one engine per GPU, node ids
split into contiguous shards, one all-gather of the exchange image per round
plus a tiny all-reduce of the stats partials.

Reference anchor: the only cross-node traffic of the reference is the
per-neighbour SyncRPC of (*NodeState).Gossip (main.go:81).  Here a round's
cross-shard traffic is a single RCCL all-gather over xGMI (torch.distributed
backend "nccl" is RCCL on ROCm); on CPU the same code runs over gloo, which is
how the N>1 path is tested without a GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.distributed as dist


class _DevPtr:
    """Zero-copy view of engine-owned device memory for torch collectives."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {
            "shape": (nbytes // 8,), "typestr": "<i8", "data": (ptr, False), "version": 3, "strides": None,
        }


def _as_tensor(ptr: int, nbytes: int, on_device: bool) -> torch.Tensor:
    if on_device:
        return torch.as_tensor(_DevPtr(ptr, nbytes), device=torch.device("cuda", torch.cuda.current_device()))
    arr = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_int64)), shape=(nbytes // 8,))
    return torch.from_numpy(arr)


def _device_collectives(group) -> bool:
    return dist.get_backend(group) == "nccl"


def sharded_round(engine, group=None) -> dict:
    """Runs one round of a sharded engine; every rank must call it."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    send_p, recv_p, nbytes = engine.exchange_buffers()
    on_dev = engine.on_device and world > 1 and _device_collectives(group)
    if world > 1:
        recv = _as_tensor(recv_p, nbytes * world, engine.on_device)
        send = _as_tensor(send_p, nbytes, engine.on_device)
        if on_dev:
            # RCCL all-gather in place: the send slice lies inside the image
            dist.all_gather_into_tensor(recv, send, group=group)
        else:
            # gloo (CPU): disjoint host buffers; device engines stage through host
            host = torch.empty(nbytes // 8 * world, dtype=torch.int64)
            dist.all_gather_into_tensor(host, send.cpu() if engine.on_device else send.clone(), group=group)
            recv.copy_(host)
            if engine.on_device:
                torch.cuda.synchronize()
    partial = engine.round_compute()
    if world > 1:
        t = torch.from_numpy(partial.view(np.int64).copy())
        if on_dev:
            t = t.cuda()
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        partial = t.cpu().numpy().view(np.uint64)
    return engine.round_commit(partial)


def sharded_run(engine, max_rounds: int, group=None) -> list:
    """Rounds until converged (same stop rule as gossip_step)."""
    if engine.on_device and torch.cuda.is_available():
        engine.set_stream(torch.cuda.current_stream().cuda_stream)
    out = []
    for _ in range(max_rounds):
        st = sharded_round(engine, group)
        out.append(st)
        if st["converged"] or (engine.cfg.mode == 0 and st["messages"] == 0):
            break
    return out
