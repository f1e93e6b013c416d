"""oracle_py.py — TEST INFRASTRUCTURE ONLY: ctypes driver of liboracle_gossip.so.

Drives the CPU restatement through the same Python wrapper class as the HIP
engine (AbiEngine), so a parity test issues identical calls to both.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "gossip-protocol_amd"))

from gossip_hip import _abi  # noqa: E402
from gossip_hip.engine import AbiEngine, make_config  # noqa: E402

LIB_PATH = os.path.join(HERE, "liboracle_gossip.so")
_LIB = None


def load_oracle() -> C.CDLL:
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: make -C oracle")
        lib = C.CDLL(LIB_PATH)
        names = [n for n, _, _ in _abi.SIGNATURES if hasattr(lib, "oracle_" + n)]
        _abi.bind(lib, "oracle_", names=set(names) - {"create"})
        lib.oracle_create.restype = C.c_int
        lib.oracle_create.argtypes = [C.POINTER(_abi.Config), C.c_int, C.POINTER(C.c_void_p)]
        lib.oracle_last_error = lambda h: b"oracle error"
        lib.oracle_peer.restype = C.c_uint32
        lib.oracle_peer.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
        lib.oracle_origin.restype = C.c_uint32
        lib.oracle_origin.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32]
        lib.oracle_philox4x32_10.restype = None
        lib.oracle_philox4x32_10.argtypes = [C.POINTER(C.c_uint32)] * 3
        _LIB = lib
    return _LIB


class OracleEngine(AbiEngine):
    """CPU restatement with the Engine interface (threads>1: OpenMP baseline)."""

    on_device = False

    def __init__(self, n_nodes, n_rumors=1, mode="push", fanout=1, seed=0, flags=0,
                 shard_rank=0, shard_count=1, threads=1, device=-1, churn_fail=0, churn_recover=0,
                 edge_loss=0, partitions=0, stall_rounds=0, params=None):
        cfg = make_config(n_nodes, n_rumors, mode, fanout, seed, flags, -1, shard_rank, shard_count,
                          churn_fail, churn_recover, edge_loss, partitions, stall_rounds)
        super().__init__(load_oracle(), "oracle_", cfg, create_extra=(C.c_int(threads),), params=params)


def philox(ctr, key):
    lib = load_oracle()
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib.oracle_philox4x32_10(c, k, o)
    return list(o)


def peer(seed, n_nodes, node, t, j):
    return int(load_oracle().oracle_peer(seed, n_nodes, node, t, j))


def origin(seed, n_nodes, r):
    return int(load_oracle().oracle_origin(seed, n_nodes, r))
