"""CPU: the C-ABI library loads, exports exactly what include/gossip.h
declares, and refuses to run without a GPU (no CPU fallback)."""
import ctypes as C
import os
import re

import pytest

import oracle_py as op
from conftest import ROOT
from gossip_hip import engine as eng_mod
from gossip_hip import _abi


def header_functions(names=("gossip.h", "gossip_shard.h")):
    src = "".join(open(os.path.join(ROOT, "include", h)).read() for h in names)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gossip_[a-z_0-9]+)\s*\(", src)))


def test_headers_split_the_contract_from_the_shard_protocol():
    """gossip.h is the drop-in contract (create, topology, inject, step, read, comm init, groups,
    timing); the per-kind steps of a host-driven sharded round live in gossip_shard.h only."""
    core, shard = set(header_functions(("gossip.h",))), set(header_functions(("gossip_shard.h",)))
    assert not core & shard
    for f in ("gossip_create", "gossip_set_topology_csr", "gossip_inject", "gossip_step", "gossip_read_bitset",
              "gossip_comm_init_rank", "gossip_group_step"):
        assert f in core, f
    for f in core | shard:
        protocol = re.match(r"gossip_(xd|cc|sparse|ae)_", f) or f.endswith("_dev") or f in (
            "gossip_exchange_buffers", "gossip_round_compute", "gossip_round_commit", "gossip_sharded_plan",
            "gossip_dense_prepare", "gossip_local_totals", "gossip_partial_len")
        assert bool(protocol) == (f in shard), f


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(eng_mod.LIB_PATH)
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    # and the Python binding covers them all
    assert {"gossip_" + n for n, _, _ in _abi.SIGNATURES} == set(names)


def test_abi_version():
    assert eng_mod.load_library().gossip_abi_version() == eng_mod._abi.ABI_VERSION == 10


def test_library_reads_no_environment():
    """Path knobs are gossip_set_param / config flags: an inherited environment variable
    cannot change a production caller's round path."""
    csrc = os.path.join(ROOT, "gossip-protocol_amd", "csrc")
    for name in os.listdir(csrc):
        src = open(os.path.join(csrc, name)).read()
        assert "getenv" not in src, name


def test_struct_layout():
    assert C.sizeof(_abi.Config) == 64
    assert C.sizeof(_abi.RoundStats) == 40


def test_host_peer_matches_oracle():
    for seed, N in [(0x5EED0001, 1 << 20), (0x5EED0003, 1 << 24), (5, 3)]:
        for n in [0, 1, N - 1, N // 2]:
            for t in range(3):
                for j in range(7):
                    assert eng_mod.peer(seed, N, n, t, j) == op.peer(seed, N, n, t, j)


def test_no_cpu_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(eng_mod.GossipError) as ei:
        eng_mod.Engine(1000, 1, "push", 3, 1)
    assert ei.value.code in (-5, -2)


def test_bad_config_rejected():
    lib = eng_mod.load_library()
    cfg = eng_mod.make_config(1, 1, "push", 3, 1)  # N < 2
    h = C.c_void_p()
    assert lib.gossip_create(C.byref(cfg), C.byref(h)) == -1
    assert b"n_nodes" in lib.gossip_last_error(None)
    cfg = eng_mod.make_config(100, 1, "push", 0, 1)  # fanout 0
    assert lib.gossip_create(C.byref(cfg), C.byref(h)) == -1
    cfg = eng_mod.make_config(100, 16, "antientropy", 1, 1, shard_count=2048)  # sharded: <= 1024 shards
    assert lib.gossip_create(C.byref(cfg), C.byref(h)) == -6
    cfg = eng_mod.make_config(100, 65, "antientropy", 1, 1)  # <= 64 components
    assert lib.gossip_create(C.byref(cfg), C.byref(h)) == -6
    cfg = eng_mod.make_config(100, 1, 7, 1, 1)  # unknown mode
    assert lib.gossip_create(C.byref(cfg), C.byref(h)) == -6
    cfg = eng_mod.make_config(100, 1, "push", 2, 1, stall_rounds=17)  # deadline out of range
    assert lib.gossip_create(C.byref(cfg), C.byref(h)) == -1


def _header_knobs():
    src = open(os.path.join(ROOT, "include", "gossip.h")).read()
    block = src[src.index("/* Knobs"):src.index("int gossip_set_param(")]
    ops, tests = block.split("Path selection", 1)
    return (set(re.findall(r'^ \*\s+"(\w+)"', ops, flags=re.M)), set(re.findall(r'^ \*\s+"(\w+)"', tests, flags=re.M)))


def test_knob_list_is_pinned():
    """gossip_set_param accepts exactly the knobs gossip.h documents: 7 operational ones and 16 that
    force the parity tests' A/B paths (round 6 removed serve_lr, serve_grid, apply_grid, push_waves
    and tile_queues, and added bin_scan_frac and replicate)."""
    ops, tests = _header_knobs()
    assert ops == {"timing", "place_tries", "ahead", "ae_ahead", "ordered_collectives", "link_gbps",
                   "rccl_dev_collectives"}
    assert tests == {"sparse_frac", "alld_frac", "sparse_direct", "mid_frac", "bin_scan_frac", "scan_queue", "filter_frac",
                     "xd_filter_frac", "xd_shards", "replicate", "cc_frac", "ae_sparse", "ae_cap", "ae_dense_bin", "ae_dense_cap",
                     "ae_dense_filter"}
    src = open(os.path.join(ROOT, "gossip-protocol_amd", "csrc", "engine.hip")).read()
    body = src[src.index("int gossip_set_param("):src.index("int gossip_set_topology_csr(")]
    assert set(re.findall(r'n == "(\w+)"', body)) == ops | tests
