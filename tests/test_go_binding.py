"""CPU: the committed Go side (gossipgpu/ cgo binding and its Maelstrom server, oracle/gossipref)
cannot drift from include/gossip.h unnoticed.  No Go toolchain exists in this image or on the GPU
box, so these checks read the Go source: every C call and constant it uses is declared in the
header, every header entry point is bound, and the config / stats field names match."""
import os
import re

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gossip.h")
SHARD_HEADER = os.path.join(ROOT, "include", "gossip_shard.h")
BINDING = os.path.join(ROOT, "gossipgpu", "gossipgpu.go")
SHARD_BINDING = os.path.join(ROOT, "gossipgpu", "gossipgpu_shard.go")


def _header(path=HEADER):
    return re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)


def _struct_fields(src, name):
    body = re.search(r"typedef struct " + name + r"\s*\{(.*?)\}", src, flags=re.S).group(1)
    return [m.group(1) for m in re.finditer(r"\b(\w+)\s*(?:\[[^\]]*\])?\s*;", body)]


def test_binding_calls_exactly_the_header_functions():
    """gossipgpu.go binds gossip.h (the drop-in contract), gossipgpu_shard.go binds gossip_shard.h
    (the per-kind steps of a host-driven sharded round), each exactly."""
    for header, binding in ((HEADER, BINDING), (SHARD_HEADER, SHARD_BINDING)):
        hdr = set(re.findall(r"\b(gossip_[a-z_0-9]+)\s*\(", _header(header)))
        go = open(binding).read()
        called = set(re.findall(r"\bC\.(gossip_[a-z_0-9]+)\s*\(", go))
        assert called <= hdr, (binding, called - hdr)
        assert called == hdr, (binding, hdr - called)  # every entry point has a Go method
    assert '#include "gossip_shard.h"' in open(SHARD_BINDING).read()


def test_binding_constants_exist():
    hdr = _header()
    go = open(BINDING).read()
    for const in set(re.findall(r"\bC\.(GOSSIP_[A-Z_0-9]+)", go)):
        assert re.search(r"\b" + const + r"\b", hdr), const
    shard = _header(SHARD_HEADER)
    for const in set(re.findall(r"\bC\.(GOSSIP_[A-Z_0-9]+)", open(SHARD_BINDING).read())):
        assert re.search(r"\b" + const + r"\b", hdr + shard), const
    assert "const ABIVersion = " + re.search(r"GOSSIP_ABI_VERSION (\d+)u", hdr).group(1) in go


def test_binding_config_and_stats_fields():
    hdr = _header()
    go = open(BINDING).read()
    cfg = _struct_fields(hdr, "gossip_config")
    lit = re.search(r"C\.gossip_config_t\{(.*?)\n\t\}", go, flags=re.S).group(1)
    assert re.findall(r"\b(\w+):\s*C\.", lit) == cfg
    stats = set(_struct_fields(hdr, "gossip_round_stats"))
    used = set(re.findall(r"\bst(?:\[i\])?\.([a-z_]+)\b", go))
    assert used and used <= stats, used - stats


def test_broadcast_server_uses_only_the_binding():
    src = open(os.path.join(ROOT, "gossipgpu", "cmd", "broadcast", "main.go")).read()
    assert 'import "C"' not in src and "maelstrom" not in src.split("import (")[1].split(")")[0]
    methods = set(re.findall(r"^func \(e \*Engine\) (\w+)\(", open(BINDING).read(), flags=re.M))
    for m in set(re.findall(r"\be\.(\w+)\(", src)):
        assert m in methods, m


def test_gossipref_covers_flood_faults_and_stall():
    """The Go restatement has the reference's own algorithm (FLOOD with the sender skip) and the
    fault / stall modes, and its test reads every golden section (tools/gossipref_transcription_check.py
    transcribes the same code line by line and runs it on the goldens)."""
    ref = open(os.path.join(ROOT, "oracle", "gossipref", "gossipref.go")).read()
    for sym in ("func (f *FloodSim) Round", "func EdgeLost", "func (s *Sim) SetFaults", "StallRounds"):
        assert sym in ref, sym
    test = open(os.path.join(ROOT, "oracle", "gossipref", "gossipref_test.go")).read()
    for sec in ("philox_kat", "peers", "origins", "random", "flood", "flood_faults", "random_faults", "antientropy"):
        assert f'`json:"{sec}"`' in test, sec
