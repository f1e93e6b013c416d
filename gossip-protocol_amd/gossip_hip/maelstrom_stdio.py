"""Maelstrom's line-delimited JSON wire format over stdio, for a whole cluster in one engine.

The reference node (main.go:99-158) is one Maelstrom process per node: the
library reads one message {"src", "dest", "body"} per stdin line and the
handlers reply on stdout.  This front-end answers for every node of a cluster
whose state lives in one engine (FLOOD mode, the reference's own algorithm):

  init       library-handled in the reference (maelstrom.NewNode, main.go:100) -> init_ok
  topology   main.go:132-149: replaces the neighbour map                       -> topology_ok
  broadcast  main.go:102-121: ack first (:109), dedupe (:113), record (:117),
             then Gossip (:118), here rounds on the engine until quiescent     -> broadcast_ok
  read       main.go:123-130                                                   -> read_ok {"messages"}
  broadcast_ok  main.go:151-153: ignored

Node-to-node gossip is internal (engine rounds), so it never appears on the
wire; its message count (the reference's msgs-per-op) is kept in `stats`.
Handler errors reply like the maelstrom Go library: code 10 (not supported)
for an unknown type, 13 (crash) for a body that does not decode
(main.go:104-106, 138-140 return the unmarshal error to the library).

    python -m gossip_hip.maelstrom_stdio < requests.jsonl

Any number of distinct values (the reference's MessageKeeper has no limit,
main.go:35-39): they fill engine pages of --page-values rumor slots each.
"""
from __future__ import annotations

import argparse
import json
import sys

from .maelstrom import Cluster

ERR_NOT_SUPPORTED = 10
ERR_CRASH = 13


class MaelstromServer:
    """Answers Maelstrom messages addressed to any node of one in-engine cluster."""

    def __init__(self, max_values: int = 0, engine_factory=None, page_values: int = 1024):
        self.max_values = max_values
        self.page_values = page_values
        self.engine_factory = engine_factory
        self.cluster: Cluster | None = None
        self.node_ids: list[str] = []
        self.topology_set = False
        self.next_msg_id = {}
        self.stats = {"broadcasts": 0, "gossip_rounds": 0, "gossip_messages": 0}

    # -- wire helpers ---------------------------------------------------------
    def _reply(self, req: dict, body: dict) -> dict:
        node = req.get("dest", "")
        mid = self.next_msg_id.get(node, 0) + 1
        self.next_msg_id[node] = mid
        out = dict(body)
        out["msg_id"] = mid
        if "msg_id" in req.get("body", {}):
            out["in_reply_to"] = req["body"]["msg_id"]
        return {"src": node, "dest": req.get("src", ""), "body": out}

    def _error(self, req: dict, code: int, text: str) -> dict:
        return self._reply(req, {"type": "error", "code": code, "text": text})

    # -- handlers -------------------------------------------------------------
    def _init(self, req: dict) -> dict:
        ids = req["body"]["node_ids"]
        if self.cluster is None:
            self.node_ids = list(ids)
            kw = {} if self.engine_factory is None else {"engine_factory": self.engine_factory}
            self.cluster = Cluster(len(ids), max_values=self.max_values, page_values=self.page_values, **kw)
            if self.cluster.ids != self.node_ids:
                raise ValueError("node_ids must be n0..n{N-1}")
        elif list(ids) != self.node_ids:
            raise ValueError("init with a different node set")
        return self._reply(req, {"type": "init_ok"})

    def _topology(self, req: dict) -> dict:
        topo = req["body"]["topology"]
        if not isinstance(topo, dict):
            raise TypeError("topology must be an object")
        # every node receives the same map (State.Topology = body.Topology, main.go:142)
        self.cluster.topology(topo)
        self.topology_set = True
        return self._reply(req, {"type": "topology_ok"})

    def _broadcast(self, req: dict) -> dict:
        msg = req["body"]["message"]
        if not isinstance(msg, int):
            raise TypeError("message must be an integer")
        reply = self._reply(req, {"type": "broadcast_ok"})  # acked before gossiping (main.go:109)
        self.stats["broadcasts"] += 1
        before = set(self.cluster.read(req["dest"]))
        self.cluster.broadcast(req["dest"], msg)
        if msg not in before:  # dedupe (main.go:113), then Gossip (:118); no topology yet: nil neighbours
            res = self.cluster.gossip()
            self.stats["gossip_rounds"] += res.rounds
            self.stats["gossip_messages"] += sum(s["messages"] for s in res.stats)
        return reply

    def _read(self, req: dict) -> dict:
        return self._reply(req, {"type": "read_ok", "messages": self.cluster.read(req["dest"])})

    def handle(self, req: dict) -> list:
        """Replies to one request (a list: zero or one message)."""
        kind = req.get("body", {}).get("type")
        if kind == "broadcast_ok":
            return []
        handlers = {"init": self._init, "topology": self._topology, "broadcast": self._broadcast,
                    "read": self._read}
        if kind not in handlers:
            return [self._error(req, ERR_NOT_SUPPORTED, f"no handler for {kind!r}")]
        if kind != "init" and self.cluster is None:
            return [self._error(req, ERR_CRASH, "node not initialised")]
        try:
            return [handlers[kind](req)]
        except (KeyError, TypeError, ValueError) as e:
            return [self._error(req, ERR_CRASH, f"{kind}: {e}")]

    def serve(self, inp=sys.stdin, out=sys.stdout) -> None:
        for line in inp:
            line = line.strip()
            if not line:
                continue
            try:
                req = json.loads(line)
            except json.JSONDecodeError as e:
                print(json.dumps({"error": f"bad json: {e}"}), file=sys.stderr)
                continue
            for rep in self.handle(req):
                out.write(json.dumps(rep) + "\n")
            out.flush()


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--max-values", type=int, default=0, help="limit on distinct broadcast values (0 = none)")
    ap.add_argument("--page-values", type=int, default=1024, help="rumor slots per engine page (<= 4096)")
    args = ap.parse_args(argv)
    MaelstromServer(args.max_values, page_values=args.page_values).serve()


if __name__ == "__main__":
    main()
