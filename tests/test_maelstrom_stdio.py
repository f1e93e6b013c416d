"""Maelstrom JSON wire format (gossip_hip.maelstrom_stdio): the reference's
handler set (main.go:102-153) answered for a whole cluster.  CPU tests drive
the oracle engine through the same front-end; the GPU test drives the HIP
engine.  Mirrors what Maelstrom's broadcast checker asserts: every
acknowledged value is in every node's read."""
import io
import json

import pytest

import oracle_py as op
from gossip_hip.maelstrom import grid_topology
from gossip_hip.maelstrom_stdio import ERR_CRASH, ERR_NOT_SUPPORTED, MaelstromServer


def _script(n, values):
    ids = [f"n{i}" for i in range(n)]
    msgs = [{"src": "c0", "dest": i, "body": {"type": "init", "msg_id": 1, "node_id": i, "node_ids": ids}}
            for i in ids]
    topo = grid_topology(n)
    msgs += [{"src": "c1", "dest": i, "body": {"type": "topology", "msg_id": 2, "topology": topo}} for i in ids]
    mid = 10
    for node, v in values:
        msgs.append({"src": "c2", "dest": node, "body": {"type": "broadcast", "message": v, "msg_id": mid}})
        mid += 1
    msgs += [{"src": "c3", "dest": i, "body": {"type": "read", "msg_id": 99}} for i in ids]
    return msgs


def _run(server, msgs):
    inp = io.StringIO("".join(json.dumps(m) + "\n" for m in msgs))
    out = io.StringIO()
    server.serve(inp, out)
    return [json.loads(line) for line in out.getvalue().splitlines()]


def _check_cluster(server, n=25):
    values = [("n0", 1000), ("n24", -7), ("n12", 42), ("n0", 1000)]  # last one: dedupe (main.go:113)
    replies = _run(server, _script(n, values))
    kinds = [r["body"]["type"] for r in replies]
    assert kinds.count("init_ok") == n and kinds.count("topology_ok") == n
    assert kinds.count("broadcast_ok") == len(values) and kinds.count("read_ok") == n
    for r in replies:
        assert "in_reply_to" in r["body"] and r["src"].startswith("n") and r["dest"].startswith("c")
    for r in replies:
        if r["body"]["type"] == "read_ok":
            assert sorted(r["body"]["messages"]) == [-7, 42, 1000]
    # three distinct values flooded over a 5x5 grid; the repeat moved nothing
    assert server.stats["broadcasts"] == 4 and server.stats["gossip_messages"] > 0
    return replies


def test_stdio_cluster_oracle():
    _check_cluster(MaelstromServer(max_values=8, engine_factory=lambda **kw: op.OracleEngine(**kw)))


def test_stdio_errors_oracle():
    s = MaelstromServer(max_values=2, engine_factory=lambda **kw: op.OracleEngine(**kw))
    out = s.handle({"src": "c", "dest": "n0", "body": {"type": "read", "msg_id": 1}})
    assert out[0]["body"]["code"] == ERR_CRASH  # not initialised
    s.handle({"src": "c", "dest": "n0", "body": {"type": "init", "msg_id": 1, "node_id": "n0",
                                                 "node_ids": ["n0", "n1"]}})
    out = s.handle({"src": "c", "dest": "n0", "body": {"type": "cas", "msg_id": 2}})
    assert out[0]["body"]["code"] == ERR_NOT_SUPPORTED and out[0]["body"]["in_reply_to"] == 2
    out = s.handle({"src": "c", "dest": "n0", "body": {"type": "broadcast", "msg_id": 3, "message": "x"}})
    assert out[0]["body"]["code"] == ERR_CRASH  # body does not decode (main.go:104-106)
    assert s.handle({"src": "n1", "dest": "n0", "body": {"type": "broadcast_ok", "in_reply_to": 5}}) == []
    for v in (1, 2):
        s.handle({"src": "c", "dest": "n1", "body": {"type": "broadcast", "msg_id": 4, "message": v}})
    out = s.handle({"src": "c", "dest": "n1", "body": {"type": "broadcast", "msg_id": 5, "message": 3}})
    assert out[0]["body"]["code"] == ERR_CRASH  # more distinct values than slots


@pytest.mark.gpu
def test_stdio_cluster_gpu():
    _check_cluster(MaelstromServer(max_values=8))


def _oracle_factory(**kw):
    return op.OracleEngine(**kw)


def test_stdio_many_values_pages_oracle():
    """A standard broadcast workload sends thousands of distinct values (the reference's
    MessageKeeper has no limit, main.go:35-39): they spill over engine pages."""
    s = MaelstromServer(engine_factory=_oracle_factory, page_values=64)
    n = 9
    values = [(f"n{i % n}", 10_000 + i) for i in range(300)]
    replies = _run(s, _script(n, values))
    assert len(s.cluster.pages) == 5  # ceil(300 / 64)
    for r in replies:
        if r["body"]["type"] == "read_ok":
            assert sorted(r["body"]["messages"]) == [v for _, v in values]
    assert [r["body"]["type"] for r in replies].count("broadcast_ok") == 300


def test_broadcast_before_topology_is_never_forwarded():
    """main.go:72 ranges over a nil Topology for a broadcast that arrives before `topology`:
    the value is recorded and acked but never forwarded, also not after the topology
    arrives; later values flood as usual."""
    n = 9
    ids = [f"n{i}" for i in range(n)]
    s = MaelstromServer(engine_factory=_oracle_factory)
    msgs = [{"src": "c0", "dest": i, "body": {"type": "init", "msg_id": 1, "node_id": i, "node_ids": ids}}
            for i in ids]
    msgs.append({"src": "c2", "dest": "n4", "body": {"type": "broadcast", "message": 5, "msg_id": 3}})
    msgs += [{"src": "c1", "dest": i, "body": {"type": "topology", "msg_id": 2, "topology": grid_topology(n)}}
             for i in ids]
    msgs.append({"src": "c2", "dest": "n0", "body": {"type": "broadcast", "message": 6, "msg_id": 4}})
    msgs += [{"src": "c3", "dest": i, "body": {"type": "read", "msg_id": 99}} for i in ids]
    reads = {r["src"]: sorted(r["body"]["messages"]) for r in _run(s, msgs) if r["body"]["type"] == "read_ok"}
    assert reads["n4"] == [5, 6]
    assert all(reads[i] == [6] for i in ids if i != "n4")
