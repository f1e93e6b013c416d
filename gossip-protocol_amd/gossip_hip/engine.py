"""Python mirror of the engine ABI (include/gossip.h).

`Engine` drives libgossip_hip.so (HIP, gfx950).  `AbiEngine` is the same
wrapper over any library exporting the ABI under another prefix; tests use it
to drive the CPU oracle with identical calls.  There is no fallback: if the
HIP library is missing or no gfx950 device exists, `Engine(...)` raises.

Reference interface mirrored (0xSherlokMo/gossip-protocol main.go):
  Engine.set_topology  ≙ topology handler, main.go:132-149
  Engine.inject        ≙ broadcast handler from a client, main.go:102-117
  Engine.step          ≙ (*NodeState).Gossip, main.go:65-89, as synchronous rounds
  Engine.read_bitset   ≙ read handler, main.go:123-130
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _abi
from ._abi import Config, RoundStats

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgossip_hip.so")
_LIB = None


class GossipError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_abi.STATUS.get(code, code)}: {msg}")
        self.code = code


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Loads libgossip_hip.so; raises if it has not been built (make -C gossip-protocol_amd)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: build it with `make -C gossip-protocol_amd` "
                                    "(the engine has no CPU fallback)")
        lib = C.CDLL(path)
        # the version first: a library of another ABI fails here with a clear message, not on the
        # first entry point it lacks
        ver = getattr(lib, "gossip_abi_version", None)
        if ver is None:
            raise RuntimeError(f"{path} exports no gossip_abi_version: not a gossip engine library")
        ver.restype = C.c_uint32
        ver.argtypes = []
        if ver() != _abi.ABI_VERSION:
            raise RuntimeError(f"{path} has ABI v{ver()}, this binding is written for v{_abi.ABI_VERSION}: "
                               "rebuild it with `make -C gossip-protocol_amd`")
        _LIB = _abi.bind(lib, "gossip_")
    return _LIB


@dataclass
class StepResult:
    rounds: int
    stats: list          # list[dict] per round
    infected: np.ndarray  # [rounds, R] uint64

    @property
    def converged(self) -> bool:
        return bool(self.stats and self.stats[-1]["converged"])


def churn_threshold(p: float) -> int:
    """Probability -> the u32 threshold x of DESIGN.md §2.7 (event iff Philox word < x)."""
    return max(0, min(0xFFFFFFFF, int(round(p * 2.0 ** 32))))


def make_config(n_nodes: int, n_rumors: int = 1, mode="push", fanout: int = 1, seed: int = 0,
                flags: int = 0, device: int = -1, shard_rank: int = 0, shard_count: int = 1,
                churn_fail: int = 0, churn_recover: int = 0, edge_loss: int = 0, partitions: int = 0,
                stall_rounds: int = 0) -> Config:
    cfg = Config()
    cfg.n_nodes = n_nodes
    cfg.n_rumors = n_rumors
    cfg.mode = _abi.MODES[mode] if isinstance(mode, str) else int(mode)
    cfg.fanout = fanout
    cfg.flags = flags
    cfg.seed = seed
    cfg.device = device
    cfg.shard_rank = shard_rank
    cfg.shard_count = shard_count
    cfg.churn_fail = churn_fail
    cfg.churn_recover = churn_recover
    cfg.edge_loss = edge_loss
    cfg.partitions = partitions
    cfg.stall_rounds = stall_rounds
    return cfg


def loss_threshold(p: float) -> int:
    """Probability -> the u32 edge_loss threshold (an edge is lost iff its Philox draw < x)."""
    return min(int(round(p * 2**32)), 2**32 - 1)


class AbiEngine:
    """Generic wrapper over a library exporting the gossip ABI under `prefix`."""

    on_device = False

    def __init__(self, lib: C.CDLL, prefix: str, cfg: Config, create_extra=(), params=None):
        self._lib, self._p = lib, prefix
        self.cfg = cfg
        h = C.c_void_p()
        rc = self._fn("create")(C.byref(cfg), *create_extra, C.byref(h))
        if rc != 0:
            raise GossipError(rc, self._fn("last_error")(None).decode(errors="replace"))
        self._h = h
        self.n_nodes = cfg.n_nodes
        self.n_rumors = cfg.n_rumors
        self.n_words = (cfg.n_rumors + 63) // 64
        lo, hi = C.c_uint64(), C.c_uint64()
        self._check(self._fn("shard_range")(self._h, C.byref(lo), C.byref(hi)))
        self.lo, self.hi = lo.value, hi.value
        for name, value in (params or {}).items():
            self.set_param(name, value)

    # -- plumbing ---------------------------------------------------------
    def _fn(self, name):
        return getattr(self._lib, self._p + name)

    def supports(self, name: str) -> bool:
        """Whether the bound library exports gossip_<name> (the CPU oracle has no sparse sharded rounds)."""
        return hasattr(self._lib, self._p + name)

    def _check(self, rc: int):
        if rc != 0:
            raise GossipError(rc, self._fn("last_error")(self._h).decode(errors="replace"))

    def close(self):
        if getattr(self, "_h", None):
            self._fn("destroy")(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- reference-shaped API ---------------------------------------------
    def set_topology(self, adjacency) -> None:
        """adjacency: list (index = node) of neighbour lists, or (row_ptr, col) arrays."""
        if isinstance(adjacency, tuple):
            row_ptr, col = (np.ascontiguousarray(a, dtype=np.uint32) for a in adjacency)
        else:
            lens = [len(r) for r in adjacency]
            row_ptr = np.zeros(len(adjacency) + 1, dtype=np.uint32)
            row_ptr[1:] = np.cumsum(lens)
            col = np.array([v for r in adjacency for v in r], dtype=np.uint32)
        colp = col if col.size else np.zeros(1, dtype=np.uint32)
        self._check(self._fn("set_topology_csr")(
            self._h, row_ptr.ctypes.data_as(_abi.U32P), colp.ctypes.data_as(_abi.U32P),
            C.c_uint64(row_ptr.size - 1), C.c_uint64(col.size)))

    def set_param(self, name: str, value: float):
        """Tuning / path-selection knob (gossip_set_param): moves time, never a result bit."""
        self._check(self._fn("set_param")(self._h, name.encode(), C.c_double(value)))

    def set_faults(self, edge_loss: int = 0, partitions: int = 0):
        """Fault model for the following rounds."""
        self._check(self._fn("set_faults")(self._h, edge_loss, partitions))

    def reset(self):
        self._check(self._fn("reset")(self._h))

    def inject(self, node: int, rumor: int = 0):
        self._check(self._fn("inject")(self._h, C.c_uint64(node), C.c_uint32(rumor)))

    def inject_random(self):
        self._check(self._fn("inject_random")(self._h))

    def step(self, max_rounds: int, with_infected: bool = True) -> StepResult:
        stats = (RoundStats * max(max_rounds, 1))()
        inf = np.zeros((max(max_rounds, 1), self.n_rumors), dtype=np.uint64) if with_infected else None
        done = C.c_uint32()
        self._check(self._fn("step")(
            self._h, C.c_uint32(max_rounds), stats,
            inf.ctypes.data_as(_abi.U64P) if inf is not None else None, C.byref(done)))
        r = done.value
        return StepResult(r, [stats[i].as_dict() for i in range(r)],
                          inf[:r] if inf is not None else np.zeros((r, 0), np.uint64))

    def read_bitset(self, node: int) -> np.ndarray:
        out = np.zeros(self.n_words, dtype=np.uint64)
        self._check(self._fn("read_bitset")(self._h, C.c_uint64(node), out.ctypes.data_as(_abi.U64P),
                                            C.c_uint32(self.n_words)))
        return out

    def read(self, node: int) -> list:
        """Rumor slots held by `node` (the read handler's view, main.go:123-130)."""
        words = self.read_bitset(node)
        return [w * 64 + b for w in range(self.n_words) for b in range(64) if (int(words[w]) >> b) & 1]

    def read_versions(self, node: int):
        """ANTIENTROPY: (versions[K], alive) of one node."""
        out = np.zeros(self.n_rumors, dtype=np.uint32)
        alive = C.c_uint32()
        self._check(self._fn("read_versions")(self._h, C.c_uint64(node), out.ctypes.data_as(_abi.U32P),
                                              C.c_uint32(self.n_rumors), C.byref(alive)))
        return out, bool(alive.value)

    def read_rows(self) -> np.ndarray:
        """ANTIENTROPY: the owned rows, [nodes, K] uint32."""
        n = self.hi - self.lo
        out = np.zeros(n * self.n_rumors, dtype=np.uint32)
        self._check(self._fn("read_rows")(self._h, out.ctypes.data_as(_abi.U32P), C.c_uint64(out.size)))
        return out.reshape(n, self.n_rumors)

    def read_shard(self) -> np.ndarray:
        n = self.hi - self.lo
        out = np.zeros(self.n_words * n, dtype=np.uint64)
        self._check(self._fn("read_shard")(self._h, out.ctypes.data_as(_abi.U64P), C.c_uint64(out.size)))
        return out.reshape(self.n_words, n)

    def state_hash(self) -> int:
        h = C.c_uint64()
        self._check(self._fn("state_hash")(self._h, C.byref(h)))
        return h.value

    @property
    def round_index(self) -> int:
        return int(self._fn("round_index")(self._h))

    # -- sharded rounds --------------------------------------
    def partial_len(self) -> int:
        return int(self._fn("partial_len")(self._h))

    def exchange_buffers(self):
        send, recv, nbytes = C.c_void_p(), C.c_void_p(), C.c_uint64()
        self._check(self._fn("exchange_buffers")(self._h, C.byref(send), C.byref(recv), C.byref(nbytes)))
        return send.value, recv.value, nbytes.value

    def dense_prepare(self):
        """Enqueues the own-slice part of a dense sharded round (no-op where the engine has none)."""
        if self.supports("dense_prepare"):
            self._check(self._fn("dense_prepare")(self._h))

    def round_compute(self) -> np.ndarray:
        out = np.zeros(self.partial_len(), dtype=np.uint64)
        self._check(self._fn("round_compute")(self._h, out.ctypes.data_as(_abi.U64P)))
        return out

    def round_commit(self, total: np.ndarray) -> dict:
        total = np.ascontiguousarray(total, dtype=np.uint64)
        st = RoundStats()
        self._check(self._fn("round_commit")(self._h, total.ctypes.data_as(_abi.U64P), C.byref(st)))
        return st.as_dict()

    # -- sparse sharded rounds (include/gossip.h; gossip_hip.sharded drives them) --
    def sharded_plan(self, total=None) -> int:
        """-1: needs global totals (local_totals + all-reduce), 0: dense round, 1: sparse round."""
        kind = C.c_int32()
        t = None if total is None else np.ascontiguousarray(total, dtype=np.uint64)
        self._check(self._fn("sharded_plan")(self._h, None if t is None else t.ctypes.data_as(_abi.U64P),
                                             C.byref(kind)))
        return kind.value

    def local_totals(self) -> np.ndarray:
        out = np.zeros(self.partial_len(), dtype=np.uint64)
        self._check(self._fn("local_totals")(self._h, out.ctypes.data_as(_abi.U64P)))
        return out

    def sparse_rare(self):
        """(device pointer, count) of this shard's rare list (16-B items)."""
        ptr, count = C.c_void_p(), C.c_uint64()
        self._check(self._fn("sparse_rare")(self._h, C.byref(ptr), C.byref(count)))
        return ptr.value, count.value

    def sparse_rare_recv(self, stride: int) -> int:
        ptr = C.c_void_p()
        self._check(self._fn("sparse_rare_recv")(self._h, stride, C.byref(ptr)))
        return ptr.value

    def sparse_scan(self, counts):
        """(device pointer, items per owner) of the push messages for other shards."""
        c = np.ascontiguousarray(counts, dtype=np.uint64)
        out = np.zeros(len(c), dtype=np.uint64)
        ptr = C.c_void_p()
        self._check(self._fn("sparse_scan")(self._h, c.ctypes.data_as(_abi.U64P), C.byref(ptr),
                                            out.ctypes.data_as(_abi.U64P)))
        return ptr.value, out

    def sparse_msg_recv(self, items: int) -> int:
        ptr = C.c_void_p()
        self._check(self._fn("sparse_msg_recv")(self._h, items, C.byref(ptr)))
        return ptr.value

    # -- sharded ANTIENTROPY (include/gossip.h gossip_ae_*; gossip_hip.sharded drives them) --
    def ae_item_words(self, which: int) -> int:
        """uint32 words of a request (0) or response (1) item, padded to 8 bytes."""
        return int(self._fn("ae_item_words")(self._h, which))

    def ae_local_target(self) -> np.ndarray:
        out = np.zeros(self.n_rumors, dtype=np.uint32)
        self._check(self._fn("ae_local_target")(self._h, out.ctypes.data_as(_abi.U32P)))
        return out

    def ae_set_target(self, target) -> None:
        t = np.ascontiguousarray(target, dtype=np.uint32)
        self._check(self._fn("ae_set_target")(self._h, t.ctypes.data_as(_abi.U32P)))

    def ae_requests(self):
        """(device pointer, items per owner) of this round's request items."""
        ptr = C.c_void_p()
        out = np.zeros(self.cfg.shard_count, dtype=np.uint64)
        self._check(self._fn("ae_requests")(self._h, C.byref(ptr), out.ctypes.data_as(_abi.U64P)))
        return ptr.value, [int(x) for x in out]

    def ae_request_recv(self, items: int) -> int:
        ptr = C.c_void_p()
        self._check(self._fn("ae_request_recv")(self._h, C.c_uint64(items), C.byref(ptr)))
        return ptr.value

    def ae_serve(self) -> int:
        ptr = C.c_void_p()
        self._check(self._fn("ae_serve")(self._h, C.byref(ptr)))
        return ptr.value

    def ae_response_recv(self) -> int:
        ptr = C.c_void_p()
        self._check(self._fn("ae_response_recv")(self._h, C.byref(ptr)))
        return ptr.value

    def ae_finish(self) -> np.ndarray:
        out = np.zeros(self.partial_len(), dtype=np.uint64)
        self._check(self._fn("ae_finish")(self._h, out.ctypes.data_as(_abi.U64P)))
        return out

    # -- exchange dense rounds (include/gossip.h gossip_xd_*; gossip_hip.sharded drives them) --
    def xd_classes(self):
        """(own bitmaps pointer, image pointer, bytes per shard): bytes > 0 when this round filters
        edges by the peer's class — all-gather bytes from every rank into the image first."""
        send, img, nb = C.c_void_p(), C.c_void_p(), C.c_uint64()
        self._check(self._fn("xd_classes")(self._h, C.byref(send), C.byref(img), C.byref(nb)))
        return send.value, img.value, int(nb.value)

    def xd_requests(self):
        """(ids pointer, values pointer, items per owner) of this round's items (uint32 ids, uint64 values)."""
        ids, vals = C.c_void_p(), C.c_void_p()
        out = np.zeros(self.cfg.shard_count, dtype=np.uint64)
        self._check(self._fn("xd_requests")(self._h, C.byref(ids), C.byref(vals), out.ctypes.data_as(_abi.U64P)))
        return ids.value, vals.value, [int(x) for x in out]

    def xd_request_recv(self, items: int):
        ids, vals = C.c_void_p(), C.c_void_p()
        self._check(self._fn("xd_request_recv")(self._h, C.c_uint64(items), C.byref(ids), C.byref(vals)))
        return ids.value, vals.value

    def xd_serve(self) -> int:
        ptr = C.c_void_p()
        self._check(self._fn("xd_serve")(self._h, C.byref(ptr)))
        return ptr.value

    def xd_response_recv(self) -> int:
        ptr = C.c_void_p()
        self._check(self._fn("xd_response_recv")(self._h, C.byref(ptr)))
        return ptr.value

    def xd_finish(self) -> np.ndarray:
        out = np.zeros(self.partial_len(), dtype=np.uint64)
        self._check(self._fn("xd_finish")(self._h, out.ctypes.data_as(_abi.U64P)))
        return out

    # -- class-coded state all-gather (include/gossip.h gossip_cc_*; gossip_hip.sharded drives them) --
    def cc_send(self):
        """(own bitmaps pointer, their bytes, own mixed words pointer, word count)."""
        bits, vals = C.c_void_p(), C.c_void_p()
        nb, n = C.c_uint64(), C.c_uint64()
        self._check(self._fn("cc_send")(self._h, C.byref(bits), C.byref(nb), C.byref(vals), C.byref(n)))
        return bits.value, nb.value, vals.value, n.value

    def cc_recv(self, stride: int):
        """(bitmap image pointer, mixed words image pointer) for stride words per shard."""
        bits, vals = C.c_void_p(), C.c_void_p()
        self._check(self._fn("cc_recv")(self._h, C.c_uint64(stride), C.byref(bits), C.byref(vals)))
        return bits.value, vals.value

    def cc_expand(self, counts) -> None:
        c = np.ascontiguousarray(counts, dtype=np.uint64)
        self._check(self._fn("cc_expand")(self._h, c.ctypes.data_as(_abi.U64P)))

    def sparse_commit(self, items: int) -> np.ndarray:
        out = np.zeros(self.partial_len(), dtype=np.uint64)
        self._check(self._fn("sparse_commit")(self._h, items, out.ctypes.data_as(_abi.U64P)))
        return out

    # -- device-resident round values (ABI v9, include/gossip.h gossip_*_dev): device pointers to
    # uint64 values that a device-side collective consumes without a host read of its own --
    def round_compute_dev(self) -> int:
        p = C.c_void_p()
        self._check(self._fn("round_compute_dev")(self._h, C.byref(p)))
        return p.value

    def sparse_rare_dev(self):
        """(rare list pointer, pointer to the count)."""
        ptr, cnt = C.c_void_p(), C.c_void_p()
        self._check(self._fn("sparse_rare_dev")(self._h, C.byref(ptr), C.byref(cnt)))
        return ptr.value, cnt.value

    def sparse_scan_dev(self, counts):
        """(messages pointer, pointer to the G items-per-owner counts)."""
        c = np.ascontiguousarray(counts, dtype=np.uint64)
        ptr, cnt = C.c_void_p(), C.c_void_p()
        self._check(self._fn("sparse_scan_dev")(self._h, c.ctypes.data_as(_abi.U64P), C.byref(ptr), C.byref(cnt)))
        return ptr.value, cnt.value

    def sparse_commit_dev(self, items: int) -> int:
        p = C.c_void_p()
        self._check(self._fn("sparse_commit_dev")(self._h, C.c_uint64(items), C.byref(p)))
        return p.value

    def xd_requests_dev(self):
        """(ids pointer, values pointer, pointer to the G items-per-owner counts)."""
        ids, vals, cnt = C.c_void_p(), C.c_void_p(), C.c_void_p()
        self._check(self._fn("xd_requests_dev")(self._h, C.byref(ids), C.byref(vals), C.byref(cnt)))
        return ids.value, vals.value, cnt.value

    def xd_finish_dev(self) -> int:
        p = C.c_void_p()
        self._check(self._fn("xd_finish_dev")(self._h, C.byref(p)))
        return p.value


class Engine(AbiEngine):
    """The HIP engine (libgossip_hip.so) on one gfx950 device."""

    on_device = True

    def __init__(self, n_nodes: int, n_rumors: int = 1, mode="push", fanout: int = 1, seed: int = 0,
                 flags: int = 0, device: int = -1, shard_rank: int = 0, shard_count: int = 1,
                 churn_fail: int = 0, churn_recover: int = 0, edge_loss: int = 0, partitions: int = 0,
                 stall_rounds: int = 0, params=None):
        cfg = make_config(n_nodes, n_rumors, mode, fanout, seed, flags, device, shard_rank, shard_count,
                          churn_fail, churn_recover, edge_loss, partitions, stall_rounds)
        super().__init__(load_library(), "gossip_", cfg, params=params)
        # None = the caller's current HIP device.  torch is not touched here: it bundles its own
        # HIP runtime, which cannot initialise after this library's in a process that did not
        # import torch first (the drivers in gossip_hip.sharded resolve None themselves)
        self.device = device if device >= 0 else None

    def set_stream(self, hip_stream: int):
        """Binds the engine to a HIP stream handle (0 = the null stream, torch's default)."""
        if getattr(self, "_stream", None) == hip_stream:
            return
        self._check(self._fn("set_stream")(self._h, C.c_void_p(hip_stream or None)))
        self._stream = hip_stream

    def comm_init_rank(self, unique_id: bytes):
        """This rank's RCCL communicator (gossip_comm_init_rank): gossip_step then runs sharded rounds."""
        self._check(self._fn("comm_init_rank")(self._h, unique_id))

    def kernel_time(self, which: int):
        ms, n = C.c_double(), C.c_uint64()
        self._check(self._fn("kernel_time")(self._h, C.c_uint32(which), C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def reset_timing(self):
        self._check(self._fn("reset_timing")(self._h))

    def round_wall(self, cls: int):
        """Library-driven sharded rounds of class cls (0 dense, 1 sparse, 2 ANTIENTROPY):
        (whole-round ms incl. collectives, rounds, link bytes this shard sent); gossip_round_wall."""
        ms, n, lb = C.c_double(), C.c_uint64(), C.c_uint64()
        self._check(self._fn("round_wall")(self._h, C.c_uint32(cls), C.byref(ms), C.byref(n), C.byref(lb)))
        return ms.value, n.value, lb.value

    def plan_model(self):
        """The planner's model of the sharded rounds it planned (gossip_plan_model): (modelled per-rank
        ms since reset_timing, its link part, rounds covered, the current run's plan string)."""
        ms, link, n = C.c_double(), C.c_double(), C.c_uint64()
        buf = C.create_string_buffer(256)
        self._check(self._fn("plan_model")(self._h, C.byref(ms), C.byref(link), C.byref(n), buf, C.c_uint32(256)))
        return ms.value, link.value, n.value, buf.value.decode()

    def philox_device(self, ctr: np.ndarray, key) -> np.ndarray:
        ctr = np.ascontiguousarray(ctr, dtype=np.uint32).reshape(-1, 4)
        key = np.ascontiguousarray(key, dtype=np.uint32)
        out = np.zeros_like(ctr)
        self._check(self._fn("philox_device")(self._h, ctr.ctypes.data_as(_abi.U32P), key.ctypes.data_as(_abi.U32P),
                                              out.ctypes.data_as(_abi.U32P), C.c_uint32(ctr.shape[0])))
        return out


def comm_unique_id() -> bytes:
    """ncclGetUniqueId through the library (rank 0; hand the bytes to every rank)."""
    lib = load_library()
    buf = C.create_string_buffer(_abi.UNIQUE_ID_BYTES)
    rc = lib.gossip_comm_unique_id(buf)
    if rc != 0:
        raise GossipError(rc, lib.gossip_last_error(None).decode(errors="replace"))
    return buf.raw


class _GroupShard(Engine):
    """Engine view of one shard of a Group (the group owns and destroys it)."""

    def __init__(self, group: "Group", handle, cfg: Config, device):
        self._lib, self._p = load_library(), "gossip_"
        self.cfg = cfg
        self._h = handle
        self._group = group
        self.n_nodes, self.n_rumors = cfg.n_nodes, cfg.n_rumors
        self.n_words = (cfg.n_rumors + 63) // 64
        lo, hi = C.c_uint64(), C.c_uint64()
        self._check(self._fn("shard_range")(self._h, C.byref(lo), C.byref(hi)))
        self.lo, self.hi = lo.value, hi.value
        self.device = device

    def close(self):  # owned by the group
        self._h = None


class Group:
    """All G shards in this process, rounds driven by the library (gossip_group_*):
    transport 1 = RCCL (distinct devices), 2 = device copies (any devices, also one GPU), 0 = auto."""

    def __init__(self, n_nodes: int, n_rumors: int = 1, mode="push", fanout: int = 1, seed: int = 0,
                 flags: int = 0, n_shards: int = 2, devices=None, transport: int = _abi.TRANSPORT_AUTO,
                 churn_fail: int = 0, churn_recover: int = 0, edge_loss: int = 0, partitions: int = 0,
                 stall_rounds: int = 0, params=None):
        self._lib = load_library()
        self.cfg = make_config(n_nodes, n_rumors, mode, fanout, seed, flags, devices[0] if devices else -1, 0,
                               n_shards, churn_fail, churn_recover, edge_loss, partitions, stall_rounds)
        devs = (C.c_int32 * n_shards)(*devices) if devices else None
        h = C.c_void_p()
        rc = self._lib.gossip_group_create(C.byref(self.cfg), n_shards, devs, transport, C.byref(h))
        if rc != 0:
            raise GossipError(rc, self._lib.gossip_group_last_error(None).decode(errors="replace"))
        self._h = h
        self.n_rumors = n_rumors
        self.shards = []
        for r in range(n_shards):
            c = Config.from_buffer_copy(self.cfg)
            c.shard_rank = r
            self.shards.append(_GroupShard(self, self._lib.gossip_group_engine(self._h, r), c,
                                           devices[r] if devices else None))
        for e in self.shards:
            for name, value in (params or {}).items():
                e.set_param(name, value)

    @property
    def transport(self) -> int:
        return self._lib.gossip_group_transport(self._h)

    def inject_random(self):
        for e in self.shards:
            e.inject_random()

    def inject(self, node: int, rumor: int = 0):
        for e in self.shards:
            e.inject(node, rumor)

    def reset(self):
        for e in self.shards:
            e.reset()

    def step(self, max_rounds: int, with_infected: bool = True) -> StepResult:
        stats = (RoundStats * max(max_rounds, 1))()
        inf = np.zeros((max(max_rounds, 1), self.n_rumors), dtype=np.uint64) if with_infected else None
        done = C.c_uint32()
        rc = self._lib.gossip_group_step(self._h, max_rounds, stats,
                                         inf.ctypes.data_as(_abi.U64P) if inf is not None else None, C.byref(done))
        if rc != 0:
            raise GossipError(rc, self._lib.gossip_group_last_error(self._h).decode(errors="replace"))
        r = done.value
        return StepResult(r, [stats[i].as_dict() for i in range(r)],
                          inf[:r] if inf is not None else np.zeros((r, 0), np.uint64))

    def close(self):
        if getattr(self, "_h", None):
            for e in self.shards:
                e.close()
            self._lib.gossip_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def peer(seed: int, n_nodes: int, node: int, round_: int, j: int) -> int:
    """p_j(node, round) as the kernels draw it (host copy of the device function)."""
    return int(load_library().gossip_peer(seed, n_nodes, node, round_, j))
