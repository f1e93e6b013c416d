"""ctypes description of include/gossip.h, shared by every binding of that ABI.

`bind(lib, prefix)` declares argument/return types for the entry points of a
library exporting the gossip ABI under `prefix` ("gossip_" for the HIP engine).
"""
from __future__ import annotations

import ctypes as C

MODE_FLOOD, MODE_PUSH, MODE_PULL, MODE_PUSHPULL, MODE_ANTIENTROPY = range(5)
MODES = {"flood": MODE_FLOOD, "push": MODE_PUSH, "pull": MODE_PULL,
         "pushpull": MODE_PUSHPULL, "antientropy": MODE_ANTIENTROPY}
FLAG_HASH = 1 << 0
FLAG_TIMING = 1 << 1
FLAG_DIRECT = 1 << 2
FLAG_DENSE = 1 << 3
FLAG_SHARD_DIRECT = 1 << 4
FLAG_AE_DIRECT_SCAN = 1 << 5

ABI_VERSION = 10  # include/gossip.h GOSSIP_ABI_VERSION (v10: gossip_round_wall)

STATUS = {0: "OK", -1: "EINVAL", -2: "EHIP", -3: "ENOMEM", -4: "ESTATE", -5: "ENODEV", -6: "ENOTSUP", -7: "ERCCL"}
UNIQUE_ID_BYTES = 128
TRANSPORT_AUTO, TRANSPORT_RCCL, TRANSPORT_COPY = 0, 1, 2


class Config(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint64),
        ("n_rumors", C.c_uint32),
        ("mode", C.c_uint32),
        ("fanout", C.c_uint32),
        ("flags", C.c_uint32),
        ("seed", C.c_uint64),
        ("device", C.c_int32),
        ("shard_rank", C.c_uint32),
        ("shard_count", C.c_uint32),
        ("churn_fail", C.c_uint32),
        ("churn_recover", C.c_uint32),
        ("edge_loss", C.c_uint32),
        ("partitions", C.c_uint32),
        ("stall_rounds", C.c_uint32),
    ]


class RoundStats(C.Structure):
    _fields_ = [
        ("round", C.c_uint32),
        ("converged", C.c_uint32),
        ("full_nodes", C.c_uint64),
        ("alive_nodes", C.c_uint64),
        ("messages", C.c_uint64),
        ("state_hash", C.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


# (name, restype, argtypes) of every entry point declared in include/gossip.h
P = C.c_void_p
U64P = C.POINTER(C.c_uint64)
U32P = C.POINTER(C.c_uint32)
SIGNATURES = [
    ("abi_version", C.c_uint32, []),
    ("create", C.c_int, [C.POINTER(Config), C.POINTER(P)]),
    ("destroy", None, [P]),
    ("last_error", C.c_char_p, [P]),
    ("set_stream", C.c_int, [P, P]),
    ("set_topology_csr", C.c_int, [P, U32P, U32P, C.c_uint64, C.c_uint64]),
    ("reset", C.c_int, [P]),
    ("inject", C.c_int, [P, C.c_uint64, C.c_uint32]),
    ("inject_random", C.c_int, [P]),
    ("set_faults", C.c_int, [P, C.c_uint32, C.c_uint32]),
    ("set_param", C.c_int, [P, C.c_char_p, C.c_double]),
    ("step", C.c_int, [P, C.c_uint32, C.POINTER(RoundStats), U64P, U32P]),
    ("partial_len", C.c_uint64, [P]),
    ("exchange_buffers", C.c_int, [P, C.POINTER(P), C.POINTER(P), U64P]),
    ("round_compute", C.c_int, [P, U64P]),
    ("dense_prepare", C.c_int, [P]),
    ("round_commit", C.c_int, [P, U64P, C.POINTER(RoundStats)]),
    ("sharded_plan", C.c_int, [P, U64P, C.POINTER(C.c_int32)]),
    ("local_totals", C.c_int, [P, U64P]),
    ("sparse_rare", C.c_int, [P, C.POINTER(P), U64P]),
    ("sparse_rare_recv", C.c_int, [P, C.c_uint64, C.POINTER(P)]),
    ("sparse_scan", C.c_int, [P, U64P, C.POINTER(P), U64P]),
    ("sparse_msg_recv", C.c_int, [P, C.c_uint64, C.POINTER(P)]),
    ("sparse_commit", C.c_int, [P, C.c_uint64, U64P]),
    ("ae_item_words", C.c_uint32, [P, C.c_uint32]),
    ("ae_local_target", C.c_int, [P, U32P]),
    ("ae_set_target", C.c_int, [P, U32P]),
    ("ae_requests", C.c_int, [P, C.POINTER(P), U64P]),
    ("ae_request_recv", C.c_int, [P, C.c_uint64, C.POINTER(P)]),
    ("ae_serve", C.c_int, [P, C.POINTER(P)]),
    ("ae_response_recv", C.c_int, [P, C.POINTER(P)]),
    ("ae_finish", C.c_int, [P, U64P]),
    ("xd_classes", C.c_int, [P, C.POINTER(P), C.POINTER(P), U64P]),
    ("xd_requests", C.c_int, [P, C.POINTER(P), C.POINTER(P), U64P]),
    ("xd_request_recv", C.c_int, [P, C.c_uint64, C.POINTER(P), C.POINTER(P)]),
    ("xd_serve", C.c_int, [P, C.POINTER(P)]),
    ("xd_response_recv", C.c_int, [P, C.POINTER(P)]),
    ("xd_finish", C.c_int, [P, U64P]),
    # device-resident round values (ABI v9): the value stays in engine memory (a uint64 pointer)
    ("round_compute_dev", C.c_int, [P, C.POINTER(P)]),
    ("sparse_rare_dev", C.c_int, [P, C.POINTER(P), C.POINTER(P)]),
    ("sparse_scan_dev", C.c_int, [P, U64P, C.POINTER(P), C.POINTER(P)]),
    ("sparse_commit_dev", C.c_int, [P, C.c_uint64, C.POINTER(P)]),
    ("xd_requests_dev", C.c_int, [P, C.POINTER(P), C.POINTER(P), C.POINTER(P)]),
    ("xd_finish_dev", C.c_int, [P, C.POINTER(P)]),
    ("cc_send", C.c_int, [P, C.POINTER(P), U64P, C.POINTER(P), U64P]),
    ("cc_recv", C.c_int, [P, C.c_uint64, C.POINTER(P), C.POINTER(P)]),
    ("cc_expand", C.c_int, [P, U64P]),
    ("read_bitset", C.c_int, [P, C.c_uint64, U64P, C.c_uint32]),
    ("read_rows", C.c_int, [P, U32P, C.c_uint64]),
    ("read_shard", C.c_int, [P, U64P, C.c_uint64]),
    ("read_versions", C.c_int, [P, C.c_uint64, U32P, C.c_uint32, U32P]),
    ("shard_range", C.c_int, [P, U64P, U64P]),
    ("state_hash", C.c_int, [P, U64P]),
    ("round_index", C.c_uint32, [P]),
    ("peer", C.c_uint32, [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]),
    ("philox_device", C.c_int, [P, U32P, U32P, U32P, C.c_uint32]),
    ("kernel_time", C.c_int, [P, C.c_uint32, C.POINTER(C.c_double), U64P]),
    ("reset_timing", C.c_int, [P]),
    ("round_wall", C.c_int, [P, C.c_uint32, C.POINTER(C.c_double), U64P, U64P]),
    ("plan_model", C.c_int, [P, C.POINTER(C.c_double), C.POINTER(C.c_double), U64P, C.c_char_p, C.c_uint32]),
    # multi-GPU driven by the engine
    ("comm_unique_id", C.c_int, [C.c_char_p]),
    ("comm_init_rank", C.c_int, [P, C.c_char_p]),
    ("group_create", C.c_int, [C.POINTER(Config), C.c_uint32, C.POINTER(C.c_int32), C.c_int32, C.POINTER(P)]),
    ("group_destroy", None, [P]),
    ("group_engine", P, [P, C.c_uint32]),
    ("group_transport", C.c_int32, [P]),
    ("group_step", C.c_int, [P, C.c_uint32, C.POINTER(RoundStats), U64P, U32P]),
    ("group_last_error", C.c_char_p, [P]),
]
# entry points of the HIP engine only (the oracle library exports the rest under "oracle_")
ENGINE_ONLY = {"comm_unique_id", "comm_init_rank", "group_create", "group_destroy", "group_engine", "group_transport",
               "group_step", "group_last_error"}


def bind(lib: C.CDLL, prefix: str, names=None) -> C.CDLL:
    for name, res, args in SIGNATURES:
        if names is not None and name not in names:
            continue
        fn = getattr(lib, prefix + name)
        fn.restype = res
        fn.argtypes = args
    return lib
