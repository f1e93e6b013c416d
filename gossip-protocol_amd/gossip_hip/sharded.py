"""Sharded rounds across ranks: one engine per GPU, node ids
split into contiguous shards.

Reference anchor: the only cross-node traffic of the reference is the
per-neighbour SyncRPC of (*NodeState).Gossip (main.go:81).  Here each round is
one of two exchanges over RCCL (torch.distributed backend "nccl" is RCCL on
ROCm; on CPU the same code runs over gloo, which is how the N>1 path is tested
without a GPU):

  dense round   all-gather of every shard's state slice (the exchange image),
                then an all-reduce of the stats partials;
  sparse round  (the engine's plan, when one class of nodes is rare) all-gather
                of each shard's rare nodes {id, value}, all-to-all of the pushes
                that land on another shard, all-reduce of the partials;
  exchange      (kind 3, DESIGN.md §5.2: dense rounds at G >= the "xd_shards" param) no
                image: all-to-all of one item per live edge {p at its owner | flags,
                S_t[n]} to p's owner, all-to-all of the pull replies back, all-reduce of
                the partials; when many nodes are empty or full, first an all-gather of
                every shard's occupancy bitmaps, so the one-way edges that move nothing
                (into an empty / full peer) are never sent;
  class-coded   (kind 4, DESIGN.md §5.1: dense rounds while few nodes are mixed) the
                state all-gather as each shard's two occupancy bitmaps (empty / full)
                plus the words of its mixed nodes, expanded into the image on arrival;
  replicated    (kinds 5 / 6, DESIGN.md §5.7: dense rounds where the links cost more than the
                extra device time, e.g. G = 2 at 2^27 nodes) every rank runs the whole round over
                the whole image in place: kind 5 after the state all-gather (as a dense round),
                kind 7 after the class-coded all-gather, kind 6 with no collective before it
                (the previous round left every node's S_{t+1} in the image); then the
                all-reduce of the own-slice partials;
  ANTIENTROPY   ("Design B") all-gather of the alive and stale bits,
                all-to-all of request items {p, n, V_t[n]} to p's owner and of its
                replies V_t[p], all-reduce of the partials; the global max vector
                by an all-reduce MAX (ncclMax) after any injection.

The engine decides the kind from the global totals it was last given, so every
rank takes the same branch.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

ITEM_WORDS = 2  # sparse exchange items are {uint64 node, uint64 value}


class _DevPtr:
    """Zero-copy view of engine-owned device memory for torch collectives."""

    def __init__(self, ptr: int, nbytes: int, width: int = 8):
        self.__cuda_array_interface__ = {
            "shape": (nbytes // width,), "typestr": f"<i{width}", "data": (ptr, False), "version": 3, "strides": None,
        }


def _as_tensor(ptr: int, nbytes: int, on_device: bool, device: int | None = None, width: int = 8) -> torch.Tensor:
    """int64 (width 8) or int32 (width 4) view of nbytes at ptr."""
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device) if on_device else "cpu"
    dt = torch.int64 if width == 8 else torch.int32
    if nbytes == 0:
        return torch.empty(0, dtype=dt, device=dev)
    if on_device:
        return torch.as_tensor(_DevPtr(ptr, nbytes, width), device=dev)
    arr = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_int64 if width == 8 else C.c_int32)),
                                shape=(nbytes // width,))
    return torch.from_numpy(arr)


def _device_collectives(group) -> bool:
    return dist.get_backend(group) == "nccl"


class _Comm:
    """The collectives a round needs, on engine memory: in place over RCCL for
    device engines, staged through host tensors over gloo."""

    def __init__(self, engine, group, direct: bool | None = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        # bytes this rank put on its links this round (the model of gossip_round_wall): an
        # all-gather sends the slice to world - 1 ranks, an all-to-all what goes to other ranks,
        # a ring all-reduce 2 (world - 1) / world of the vector
        self.link = 0
        self.on_device = engine.on_device
        self.direct = engine.on_device and self.world > 1 and _device_collectives(group)
        if direct is not None:  # tests: the collectives on engine memory as RCCL would run them
            self.direct = direct and self.world > 1

    def _sync(self):
        if self.on_device:
            torch.cuda.synchronize()

    def _lb_gather(self, send: torch.Tensor):
        self.link += send.numel() * send.element_size() * (self.world - 1)

    def _lb_a2a(self, send: torch.Tensor, send_splits):
        el = send.element_size()
        self.link += sum(int(c) * el for q, c in enumerate(send_splits) if q != self.rank)

    def _lb_reduce(self, t: torch.Tensor):
        self.link += 2 * (self.world - 1) * t.numel() * t.element_size() // max(self.world, 1)

    def all_gather(self, recv: torch.Tensor, send: torch.Tensor):
        self._lb_gather(send)
        if self.direct:
            dist.all_gather_into_tensor(recv, send, group=self.group)
            return
        host = torch.empty(recv.numel(), dtype=torch.int64)
        dist.all_gather_into_tensor(host, send.cpu() if self.on_device else send.clone(), group=self.group)
        recv.copy_(host)
        self._sync()

    def all_gather_async(self, recv: torch.Tensor, send: torch.Tensor):
        """Device collectives: returns the pending work (the caller's stream waits on wait());
        staged collectives complete before returning None."""
        if self.direct:
            self._lb_gather(send)
            return dist.all_gather_into_tensor(recv, send, group=self.group, async_op=True)
        self.all_gather(recv, send)
        return None

    def all_to_all(self, recv: torch.Tensor, send: torch.Tensor, recv_splits, send_splits):
        self._lb_a2a(send, send_splits)
        if self.direct:
            dist.all_to_all_single(recv, send, output_split_sizes=recv_splits, input_split_sizes=send_splits,
                                   group=self.group)
            return
        host = torch.empty(recv.numel(), dtype=recv.dtype)
        dist.all_to_all_single(host, send.cpu() if self.on_device else send.clone(), output_split_sizes=recv_splits,
                               input_split_sizes=send_splits, group=self.group)
        recv.copy_(host)
        self._sync()

    def small(self, values) -> torch.Tensor:
        t = torch.as_tensor(np.asarray(values, dtype=np.int64).copy())
        return t.cuda() if self.direct and self.on_device else t

    def all_reduce_max(self, values: np.ndarray) -> np.ndarray:
        t = self.small(np.asarray(values, dtype=np.int64))
        self._lb_reduce(t)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t.cpu().numpy()

    def all_reduce_sum(self, partial: np.ndarray) -> np.ndarray:
        t = self.small(partial.view(np.int64))
        self._lb_reduce(t)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t.cpu().numpy().view(np.uint64)

    def all_gather_small(self, value: int) -> list:
        self.link += 8 * (self.world - 1)
        out = self.small(np.zeros(self.world))
        dist.all_gather_into_tensor(out, self.small([value]), group=self.group)
        return [int(x) for x in out.cpu()]

    def all_to_all_small(self, values) -> list:
        self.link += 8 * (self.world - 1)
        out = self.small(np.zeros(self.world))
        dist.all_to_all_single(out, self.small(values), group=self.group)
        return [int(x) for x in out.cpu()]

    # device-resident values (engine.*_dev, RCCL): the collective reads engine memory on the
    # engine's (= torch's current) stream and one host read of its result is the round's only
    # sync for that exchange
    def dev_all_gather_one(self, ptr: int) -> list:
        self.link += 8 * (self.world - 1)
        out = torch.empty(self.world, dtype=torch.int64, device="cuda")
        dist.all_gather_into_tensor(out, _as_tensor(ptr, 8, True), group=self.group)
        return [int(x) for x in out.cpu()]

    def dev_all_to_all_counts(self, ptr: int):
        """(sent counts, received counts) from the G counts at ptr."""
        send = _as_tensor(ptr, self.world * 8, True)
        self.link += 8 * (self.world - 1)
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=self.group)
        both = [int(x) for x in torch.cat([send, recv]).cpu()]
        return both[:self.world], both[self.world:]

    def dev_all_reduce_sum(self, ptr: int, n: int) -> np.ndarray:
        t = _as_tensor(ptr, n * 8, True).clone()  # (the engine keeps its own partials)
        self._lb_reduce(t)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t.cpu().numpy().view(np.uint64)


def _dev_values(engine, comm: "_Comm") -> bool:
    """Device-side counts and partials (RCCL on device engines with the ABI v9 calls)."""
    return comm.direct and engine.on_device and comm.world > 1 and engine.supports("round_compute_dev")


def _plan(engine, comm: _Comm) -> int:
    if not engine.supports("sharded_plan"):
        return 0
    kind = engine.sharded_plan()
    if kind == -2:  # ANTIENTROPY: the global max vector after an injection (ncclMax over the shards)
        t = engine.ae_local_target()
        engine.ae_set_target(comm.all_reduce_max(t) if comm.world > 1 else t)
        kind = engine.sharded_plan()
    if kind < 0:  # no global totals yet (after reset / inject): all-reduce the shards' own
        kind = engine.sharded_plan(comm.all_reduce_sum(engine.local_totals()) if comm.world > 1
                                   else engine.local_totals())
    return kind


def _dense_round(engine, comm: _Comm) -> np.ndarray:
    send_p, recv_p, nbytes = engine.exchange_buffers()
    if comm.world > 1:
        recv = _as_tensor(recv_p, nbytes * comm.world, engine.on_device)
        send = _as_tensor(send_p, nbytes, engine.on_device)
        # RCCL all-gather in place (the send slice lies inside the image), in flight
        # while the engine runs the part of the round that reads only its own slice
        work = comm.all_gather_async(recv, send)
        engine.dense_prepare()
        if work is not None:
            work.wait()
    if _dev_values(engine, comm):
        return comm.dev_all_reduce_sum(engine.round_compute_dev(), engine.partial_len())
    return engine.round_compute()


def _sparse_round(engine, comm: _Comm) -> np.ndarray:
    w = comm.world
    dev = _dev_values(engine, comm)
    if dev:
        send_p, count_p = engine.sparse_rare_dev()
        counts = comm.dev_all_gather_one(count_p)
    else:
        send_p, count = engine.sparse_rare()
        counts = comm.all_gather_small(count)
    stride = max(counts)
    recv_p = engine.sparse_rare_recv(stride)
    if stride:
        comm.all_gather(_as_tensor(recv_p, stride * 16 * w, engine.on_device),
                        _as_tensor(send_p, stride * 16, engine.on_device))
    if dev:
        out_p, counts_p = engine.sparse_scan_dev(counts)
        out_counts, in_counts = comm.dev_all_to_all_counts(counts_p)
    else:
        out_p, out_counts = engine.sparse_scan(counts)
        out_counts = [int(c) for c in out_counts]
        in_counts = comm.all_to_all_small(out_counts)
    n_in = sum(in_counts)
    in_p = engine.sparse_msg_recv(n_in)
    # every rank joins the collective, also one with nothing to send or receive (G > 2)
    comm.all_to_all(_as_tensor(in_p, n_in * 16, engine.on_device),
                    _as_tensor(out_p, sum(out_counts) * 16, engine.on_device),
                    [c * ITEM_WORDS for c in in_counts], [c * ITEM_WORDS for c in out_counts])
    if dev:
        return comm.dev_all_reduce_sum(engine.sparse_commit_dev(n_in), engine.partial_len())
    return engine.sparse_commit(n_in)


def _xd_round(engine, comm: _Comm) -> np.ndarray:
    cls_p, img_p, nb = engine.xd_classes()
    if nb and comm.world > 1:  # every shard's class bitmaps (in place): the edge filter of this round
        comm.all_gather(_as_tensor(img_p, nb * comm.world, engine.on_device), _as_tensor(cls_p, nb, engine.on_device))
    dv = _dev_values(engine, comm)
    if dv:
        ids_p, vals_p, counts_p = engine.xd_requests_dev()
        counts, in_counts = comm.dev_all_to_all_counts(counts_p)
    else:
        ids_p, vals_p, counts = engine.xd_requests()
        in_counts = comm.all_to_all_small(counts) if comm.world > 1 else counts
    n_in, n_out = sum(in_counts), sum(counts)
    rid_p, rval_p = engine.xd_request_recv(n_in)
    dev = engine.on_device
    if comm.world > 1:
        comm.all_to_all(_as_tensor(rid_p, n_in * 4, dev, width=4), _as_tensor(ids_p, n_out * 4, dev, width=4),
                        in_counts, counts)
        comm.all_to_all(_as_tensor(rval_p, n_in * 8, dev), _as_tensor(vals_p, n_out * 8, dev), in_counts, counts)
    else:
        _as_tensor(rid_p, n_in * 4, dev, width=4).copy_(_as_tensor(ids_p, n_out * 4, dev, width=4))
        _as_tensor(rval_p, n_in * 8, dev).copy_(_as_tensor(vals_p, n_out * 8, dev))
    rep_p = engine.xd_serve()  # replies in the received order
    back_p = engine.xd_response_recv()
    if comm.world > 1:
        comm.all_to_all(_as_tensor(back_p, n_out * 8, dev), _as_tensor(rep_p, n_in * 8, dev), counts, in_counts)
    else:
        _as_tensor(back_p, n_out * 8, dev).copy_(_as_tensor(rep_p, n_in * 8, dev))
    if dv:
        return comm.dev_all_reduce_sum(engine.xd_finish_dev(), engine.partial_len())
    return engine.xd_finish()


def _rep_round(engine, comm: _Comm) -> np.ndarray:
    """Kind 6: the image already holds S_t of every node (the last round was replicated)."""
    if _dev_values(engine, comm):
        return comm.dev_all_reduce_sum(engine.round_compute_dev(), engine.partial_len())
    return engine.round_compute()


def _cc_round(engine, comm: _Comm) -> np.ndarray:
    bits_p, nbytes, vals_p, count = engine.cc_send()
    w, dev = comm.world, engine.on_device
    counts = comm.all_gather_small(count) if w > 1 else [count]
    stride = max(counts)
    img_p, rvals_p = engine.cc_recv(stride)
    if w > 1:
        # the bitmaps in place (the own slot lies inside the image); the mixed words padded to
        # the stride.  Both in flight while the engine runs the own-slice part of the round.
        works = [comm.all_gather_async(_as_tensor(img_p, nbytes * w, dev), _as_tensor(bits_p, nbytes, dev))]
        if stride:
            works.append(comm.all_gather_async(_as_tensor(rvals_p, stride * 8 * w, dev),
                                               _as_tensor(vals_p, stride * 8, dev)))
        engine.dense_prepare()
        for work in works:
            if work is not None:
                work.wait()
    elif count:
        _as_tensor(rvals_p, count * 8, dev).copy_(_as_tensor(vals_p, count * 8, dev))
    engine.cc_expand(counts)
    if _dev_values(engine, comm):
        return comm.dev_all_reduce_sum(engine.round_compute_dev(), engine.partial_len())
    return engine.round_compute()


def _bind_stream(engine, comm: _Comm) -> bool:
    """Device collectives are enqueued on torch's current stream (the RCCL stream waits for
    it, and work.wait() / a synchronous collective make it wait in turn): the engine must
    launch on that same stream, or its kernels could read the image before the all-gather
    wrote it.  torch's default stream is the null stream (cuda_stream 0), which
    gossip_set_stream binds as such.  Returns True when it also set ordered_collectives (torch's
    collectives wait for this stream, so the per-kind calls skip their publishing sync); the
    caller clears it when the round ends (sharded_round), so the flag never outlives the round
    that bound the stream (a later host driver, staged collectives or another stream get the
    sync back)."""
    if comm.direct and comm.on_device:
        engine.set_stream(torch.cuda.current_stream().cuda_stream)
        engine.set_param("ordered_collectives", 1)
        return True
    return False


def _ae_round(engine, comm: _Comm) -> np.ndarray:
    w = comm.world
    rw, pw = engine.ae_item_words(0), engine.ae_item_words(1)  # uint32 words, even: whole int64s
    send_p, recv_p, nbytes = engine.exchange_buffers()  # own stale words -> every shard's image
    if w > 1:
        comm.all_gather(_as_tensor(recv_p, nbytes * w, engine.on_device), _as_tensor(send_p, nbytes, engine.on_device))
    req_p, counts = engine.ae_requests()
    in_counts = comm.all_to_all_small(counts) if w > 1 else counts
    n_in = sum(in_counts)
    in_p = engine.ae_request_recv(n_in)
    if w > 1:  # (every rank joins, also one with nothing to send or receive)
        comm.all_to_all(_as_tensor(in_p, n_in * rw * 4, engine.on_device),
                        _as_tensor(req_p, sum(counts) * rw * 4, engine.on_device),
                        [c * rw // 2 for c in in_counts], [c * rw // 2 for c in counts])
    resp_p = engine.ae_serve()  # replies in the received order
    back_p = engine.ae_response_recv()
    if w > 1:
        comm.all_to_all(_as_tensor(back_p, sum(counts) * pw * 4, engine.on_device),
                        _as_tensor(resp_p, n_in * pw * 4, engine.on_device),
                        [c * pw // 2 for c in counts], [c * pw // 2 for c in in_counts])
    return engine.ae_finish()


def sharded_round(engine, group=None, kinds: list | None = None, direct: bool | None = None,
                  trace: list | None = None) -> dict:
    """Runs one round of a sharded engine; every rank must call it.  With RCCL the engine is
    bound to the caller's current torch stream, so every kernel is ordered after the
    collectives that feed it.  kinds: the round's plan kind is appended to it.  direct (tests):
    force the in-place collective path that RCCL takes, also for host engines over gloo.
    trace: gets {"kind", "link_bytes"} of the round (the bytes this rank sent over its links)."""
    comm = _Comm(engine, group, direct)
    ordered = _bind_stream(engine, comm)
    try:
        kind = _plan(engine, comm)
        if kinds is not None:
            kinds.append(kind)
        if kind == 2:
            partial = _ae_round(engine, comm)
        elif kind == 3:
            partial = _xd_round(engine, comm)
        elif kind in (4, 7):  # 7: the class-coded all-gather, then the replicated round
            partial = _cc_round(engine, comm)
        elif kind == 1:
            partial = _sparse_round(engine, comm)
        elif kind == 6:
            partial = _rep_round(engine, comm)
        else:  # 0, and 5 (the state all-gather, then the replicated round)
            partial = _dense_round(engine, comm)
        # the device-value path returns the global sum already (one all-reduce on engine memory)
        if comm.world > 1 and not (kind != 2 and _dev_values(engine, comm)):
            partial = comm.all_reduce_sum(partial)
        st = engine.round_commit(partial)
        if trace is not None:
            trace.append({"kind": kind, "link_bytes": comm.link})
        return st
    finally:
        if ordered:  # scoped to this round (the flag must not outlive the binding)
            engine.set_param("ordered_collectives", 0)


def _all_ranks(ok: bool, group=None) -> bool:
    """True iff `ok` holds on every rank (an all-reduce MIN: every rank learns the same answer)."""
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def init_engine_comm(engine, group=None) -> str | None:
    """Hands a shard engine its own RCCL communicator (gossip_comm_init_rank): rank 0
    makes the unique id, torch.distributed carries it; engine.step then runs every sharded round
    inside the library (plan, collectives on the engine's stream, kernels).

    Collective, and so is its outcome: every rank joins every step, also after a failure, and
    every rank returns the same thing — None when every rank has its communicator, else the
    reason (then the caller drives the rounds over torch.distributed on every rank).  Rank 0
    broadcasts the id or None; each rank first loads RCCL itself (a rank that could not would
    leave the others waiting inside ncclCommInitRank), and the init's success is agreed on by
    an all-reduce MIN."""
    from .engine import comm_unique_id
    rank0 = dist.get_rank(group) == 0
    box, err = [None], None
    try:  # rank 0: the id; every rank: RCCL loads and answers (a throwaway id elsewhere)
        uid = comm_unique_id()
        if rank0:
            box[0] = uid
    except Exception as exc:  # noqa: BLE001 - reported in the return value
        err = f"RCCL unavailable on rank {dist.get_rank(group)}: {exc}"
    dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    if not _all_ranks(err is None and box[0] is not None, group):
        return err or "RCCL unavailable on another rank"
    try:
        engine.comm_init_rank(box[0])
    except Exception as exc:  # noqa: BLE001
        err = f"gossip_comm_init_rank on rank {dist.get_rank(group)}: {exc}"
    if not _all_ranks(err is None, group):
        return err or "gossip_comm_init_rank failed on another rank"
    return None


def sharded_run(engine, max_rounds: int, group=None, kinds: list | None = None, direct: bool | None = None,
                trace: list | None = None) -> list:
    """Rounds until converged (same stop rule as gossip_step); kinds collects the plan kinds.
    trace: one entry per round, {"kind", "link_bytes"} and, on a device engine, "events" = a
    timing torch.cuda.Event pair on the current stream around the whole round (plan,
    collectives, kernels, host reads: the RCCL collectives are ordered on that stream)."""
    on_dev = engine.on_device and torch.cuda.is_available()
    if on_dev:
        engine.set_stream(torch.cuda.current_stream().cuda_stream)
    out = []
    for _ in range(max_rounds):
        ev = None
        if trace is not None and on_dev:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        st = sharded_round(engine, group, kinds, direct, trace)
        if ev is not None:
            ev[1].record()
            trace[-1]["events"] = ev
        out.append(st)
        if st["converged"] or (engine.cfg.mode == 0 and st["messages"] == 0):
            break
    return out


# -- single-process driver ---------------------------------------------------

def _sync_all(engines):
    for d in {e.device for e in engines if e.on_device}:
        torch.cuda.synchronize(d)


def _lockstep_sum(parts):
    tot = np.zeros_like(parts[0])
    for p in parts:
        tot = tot + p  # uint64 wraps like the RCCL int64 sum
    return tot


def _lockstep_dense(engines):
    G = len(engines)
    bufs = [e.exchange_buffers() for e in engines]
    for e in engines:  # on the engines' streams, concurrent with the copies below (disjoint slices)
        e.dense_prepare()
    for e, (_, recv_p, nbytes) in zip(engines, bufs):
        recv = _as_tensor(recv_p, nbytes * G, True, e.device)
        for q, (send_q, _, _) in enumerate(bufs):
            if engines[q] is not e:
                recv[q * nbytes // 8:(q + 1) * nbytes // 8].copy_(_as_tensor(send_q, nbytes, True, engines[q].device))
    _sync_all(engines)
    return [e.round_compute() for e in engines]


def _lockstep_sparse(engines):
    G = len(engines)
    rare = [e.sparse_rare() for e in engines]
    counts = [c for _, c in rare]
    stride = max(counts)
    recvs = [e.sparse_rare_recv(stride) for e in engines]
    if stride:
        for e, rp in zip(engines, recvs):
            recv = _as_tensor(rp, stride * 16 * G, True, e.device)
            for q, (sp, _) in enumerate(rare):
                recv[q * stride * ITEM_WORDS:(q + 1) * stride * ITEM_WORDS].copy_(
                    _as_tensor(sp, stride * 16, True, engines[q].device))
        _sync_all(engines)
    scans = [e.sparse_scan(counts) for e in engines]
    outs = [(p, [int(c) for c in cnt]) for p, cnt in scans]
    n_in = [sum(outs[q][1][r] for q in range(G)) for r in range(G)]
    ins = [e.sparse_msg_recv(n) for e, n in zip(engines, n_in)]
    for r in range(G):
        dst = _as_tensor(ins[r], n_in[r] * 16, True, engines[r].device)
        at = 0
        for q, (sp, cnt) in enumerate(outs):
            off = sum(cnt[:r])
            if cnt[r]:
                src = _as_tensor(sp, sum(cnt) * 16, True, engines[q].device)
                dst[at * ITEM_WORDS:(at + cnt[r]) * ITEM_WORDS].copy_(src[off * ITEM_WORDS:(off + cnt[r]) * ITEM_WORDS])
                at += cnt[r]
    _sync_all(engines)
    return [e.sparse_commit(n) for e, n in zip(engines, n_in)]


def _lockstep_ae(engines):
    G = len(engines)
    rw, pw = engines[0].ae_item_words(0), engines[0].ae_item_words(1)
    bufs = [e.exchange_buffers() for e in engines]
    for e, (_, recv_p, nbytes) in zip(engines, bufs):  # all-gather of the stale words
        recv = _as_tensor(recv_p, nbytes * G, True, e.device)
        for q, (send_q, _, _) in enumerate(bufs):
            if engines[q] is not e:
                recv[q * nbytes // 8:(q + 1) * nbytes // 8].copy_(_as_tensor(send_q, nbytes, True, engines[q].device))
    _sync_all(engines)
    reqs = [e.ae_requests() for e in engines]  # (ptr, counts[owner])
    n_in = [sum(reqs[q][1][r] for q in range(G)) for r in range(G)]
    inbox = [e.ae_request_recv(n) for e, n in zip(engines, n_in)]
    w64 = rw // 2
    for r in range(G):  # all-to-all: owner r receives from q = 0..G-1 in order
        dst = _as_tensor(inbox[r], n_in[r] * rw * 4, True, engines[r].device)
        at = 0
        for q, (rp, cnt) in enumerate(reqs):
            if cnt[r]:
                src = _as_tensor(rp, sum(cnt) * rw * 4, True, engines[q].device)
                off = sum(cnt[:r])
                dst[at * w64:(at + cnt[r]) * w64].copy_(src[off * w64:(off + cnt[r]) * w64])
                at += cnt[r]
    _sync_all(engines)
    resp = [e.ae_serve() for e in engines]
    back = [e.ae_response_recv() for e in engines]
    p64 = pw // 2
    for q, (_, cnt) in enumerate(reqs):  # replies return to requester q in its request order
        dst = _as_tensor(back[q], sum(cnt) * pw * 4, True, engines[q].device)
        at = 0
        for r in range(G):
            if cnt[r]:
                src = _as_tensor(resp[r], n_in[r] * pw * 4, True, engines[r].device)
                start = sum(reqs[q2][1][r] for q2 in range(q))  # where q's items landed in r's inbox
                dst[at * p64:(at + cnt[r]) * p64].copy_(src[start * p64:(start + cnt[r]) * p64])
                at += cnt[r]
    _sync_all(engines)
    return [e.ae_finish() for e in engines]


def _lockstep_xd(engines, items: list | None = None):
    """Exchange round of G engines in one process (device or host engines: copies in place of the
    collectives); items gets each shard's per-owner item counts."""
    G = len(engines)

    def view(e, ptr, nbytes, width=8):
        return _as_tensor(ptr, nbytes, e.on_device, e.device if e.on_device else None, width=width)

    cls = [e.xd_classes() for e in engines]
    if cls[0][2]:  # the class bitmaps of every shard into every image (the own slot is in place)
        nb = cls[0][2]
        for e, (_, img_p, _) in zip(engines, cls):
            img = view(e, img_p, nb * G)
            for q, (send_q, _, _) in enumerate(cls):
                if engines[q] is not e:
                    img[q * nb // 8:(q + 1) * nb // 8].copy_(view(engines[q], send_q, nb))
        _sync_all(engines)
    reqs = [e.xd_requests() for e in engines]  # (ids, vals, counts[owner])
    if items is not None:
        items.append([list(r[2]) for r in reqs])
    n_in = [sum(reqs[q][2][r] for q in range(G)) for r in range(G)]
    inbox = [e.xd_request_recv(n) for e, n in zip(engines, n_in)]
    for r in range(G):  # all-to-all: owner r receives from q = 0..G-1 in order
        di = view(engines[r], inbox[r][0], n_in[r] * 4, width=4)
        dv = view(engines[r], inbox[r][1], n_in[r] * 8)
        at = 0
        for q, (ip, vp, cnt) in enumerate(reqs):
            if cnt[r]:
                off, tot = sum(cnt[:r]), sum(cnt)
                si = view(engines[q], ip, tot * 4, width=4)
                sv = view(engines[q], vp, tot * 8)
                di[at:at + cnt[r]].copy_(si[off:off + cnt[r]])
                dv[at:at + cnt[r]].copy_(sv[off:off + cnt[r]])
                at += cnt[r]
    _sync_all(engines)
    reps = [e.xd_serve() for e in engines]
    back = [e.xd_response_recv() for e in engines]
    for q, (_, _, cnt) in enumerate(reqs):  # replies return to q in its send order
        dst = view(engines[q], back[q], sum(cnt) * 8)
        at = 0
        for r in range(G):
            if cnt[r]:
                src = view(engines[r], reps[r], n_in[r] * 8)
                start = sum(reqs[q2][2][r] for q2 in range(q))  # where q's items landed in r's inbox
                dst[at:at + cnt[r]].copy_(src[start:start + cnt[r]])
                at += cnt[r]
    _sync_all(engines)
    return [e.xd_finish() for e in engines]


def _lockstep_cc(engines):
    G = len(engines)
    sends = [e.cc_send() for e in engines]  # (bits, bits bytes, mixed words, count)
    counts = [c for _, _, _, c in sends]
    stride = max(counts)
    recvs = [e.cc_recv(stride) for e in engines]
    for e in engines:  # the own-slice part, on the engines' streams
        e.dense_prepare()
    for e, (img_p, vals_p) in zip(engines, recvs):
        nb = sends[0][1]
        img = _as_tensor(img_p, nb * G, True, e.device)
        vals = _as_tensor(vals_p, stride * 8 * G, True, e.device)
        for q, (bp, _, sp, _) in enumerate(sends):
            if engines[q] is not e:
                img[q * nb // 8:(q + 1) * nb // 8].copy_(_as_tensor(bp, nb, True, engines[q].device))
            if stride:
                vals[q * stride:(q + 1) * stride].copy_(_as_tensor(sp, stride * 8, True, engines[q].device))
    _sync_all(engines)
    for e in engines:
        e.cc_expand(counts)
    return [e.round_compute() for e in engines]


def lockstep_run(engines, max_rounds: int, items: list | None = None):
    """One process driving G shard engines (one per GPU, or several on one) through the
    same rounds as sharded_run, with device copies in place of the collectives.
    Returns (per-round stats, per-round kind: 0 dense / 1 sparse / 2 ANTIENTROPY / 3 exchange dense /
    4 class-coded dense / 5, 7, 6 replicated dense after the all-gather, after the class-coded one, or
    without any).  items (exchange rounds; host engines too): per round, each shard's
    item counts per owner."""
    stats, kinds = [], []
    for _ in range(max_rounds):
        ks = [e.sharded_plan() for e in engines]
        if ks[0] == -2:  # ANTIENTROPY: global max vector = elementwise max of the shards' (ncclMax)
            t = np.maximum.reduce([e.ae_local_target() for e in engines])
            for e in engines:
                e.ae_set_target(t)
            ks = [e.sharded_plan() for e in engines]
        if ks[0] == -1:
            tot = _lockstep_sum([e.local_totals() for e in engines])
            ks = [e.sharded_plan(tot) for e in engines]
        assert len(set(ks)) == 1
        kinds.append(ks[0])
        if ks[0] == 3:
            parts = _lockstep_xd(engines, items)
        else:
            parts = {1: _lockstep_sparse, 2: _lockstep_ae, 4: _lockstep_cc, 7: _lockstep_cc,
                     6: lambda es: [e.round_compute() for e in es]}.get(ks[0], _lockstep_dense)(engines)
        tot = _lockstep_sum(parts)
        st = [e.round_commit(tot) for e in engines]
        assert all(s == st[0] for s in st)
        stats.append(st[0])
        if st[0]["converged"]:
            break
    return stats, kinds
