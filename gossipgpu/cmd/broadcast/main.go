// Command broadcast answers Maelstrom's broadcast workload for a whole cluster held in one
// MI355X engine: line-delimited JSON on stdin/stdout, the handler set of the reference node
// (0xSherlokMo/gossip-protocol main.go:99-158) — init, topology, broadcast, read, and
// broadcast_ok ignored — for every node id of the cluster instead of one process per node.
//
// Node-to-node gossip happens as FLOOD rounds on the engine (the restatement of
// (*NodeState).Gossip, main.go:65-89), not on the wire.  Distinct values fill engine pages of
// -page-values rumor slots (the reference's MessageKeeper has no limit, main.go:35-39).  A
// broadcast that arrives before the topology is recorded and never forwarded, as the reference
// ranges over a nil Topology (main.go:72).  gossip-protocol_amd/gossip_hip/maelstrom_stdio.py
// is the same server in Python (tested there against the CPU oracle and the GPU engine).
package main

import (
	"bufio"
	"encoding/json"
	"flag"
	"fmt"
	"os"

	"gossipgpu"
)

const (
	errNotSupported = 10 // maelstrom error codes, as the Go library replies to handler errors
	errCrash        = 13
)

type envelope struct {
	Src  string          `json:"src"`
	Dest string          `json:"dest"`
	Body json.RawMessage `json:"body"`
}

type server struct {
	ids        []string
	pageValues uint32
	pages      []*gossipgpu.Engine
	slotOf     map[int64]uint32 // value -> slot   (MessageKeeper.broadcasted, main.go:24)
	values     []int64          // slot -> value   (MessageKeeper.messages, main.go:23)
	topo       map[string][]string
	msgID      map[string]int64
	out        *bufio.Writer
	rounds     uint64
	messages   uint64
}

func (s *server) reply(req envelope, body map[string]any) {
	var in struct {
		MsgID *int64 `json:"msg_id"`
	}
	_ = json.Unmarshal(req.Body, &in)
	s.msgID[req.Dest]++
	body["msg_id"] = s.msgID[req.Dest]
	if in.MsgID != nil {
		body["in_reply_to"] = *in.MsgID
	}
	b, _ := json.Marshal(map[string]any{"src": req.Dest, "dest": req.Src, "body": body})
	s.out.Write(append(b, '\n'))
}

func (s *server) fail(req envelope, code int, text string) {
	s.reply(req, map[string]any{"type": "error", "code": code, "text": text})
}

func (s *server) newPage() (*gossipgpu.Engine, error) {
	e, err := gossipgpu.New(gossipgpu.Config{Nodes: uint64(len(s.ids)), Rumors: s.pageValues, Mode: gossipgpu.Flood,
		Device: -1, ShardCount: 1})
	if err != nil {
		return nil, err
	}
	if s.topo != nil {
		err = e.SetTopologyMap(s.topo)
	} else { // an empty neighbour map until the topology message arrives
		err = e.SetTopology(make([]uint32, len(s.ids)+1), nil)
	}
	if err != nil {
		e.Close()
		return nil, err
	}
	s.pages = append(s.pages, e)
	return e, nil
}

func (s *server) handle(req envelope) error {
	var head struct {
		Type string `json:"type"`
	}
	if err := json.Unmarshal(req.Body, &head); err != nil {
		s.fail(req, errCrash, err.Error())
		return nil
	}
	if head.Type != "init" && head.Type != "broadcast_ok" && s.pages == nil {
		s.fail(req, errCrash, "node not initialised")
		return nil
	}
	switch head.Type {
	case "init":
		var b struct {
			NodeIDs []string `json:"node_ids"`
		}
		if err := json.Unmarshal(req.Body, &b); err != nil {
			s.fail(req, errCrash, err.Error())
			return nil
		}
		if s.pages == nil {
			for i, id := range b.NodeIDs {
				if id != fmt.Sprintf("n%d", i) {
					s.fail(req, errCrash, "node_ids must be n0..n{N-1}")
					return nil
				}
			}
			s.ids = b.NodeIDs
			if _, err := s.newPage(); err != nil {
				return err
			}
		}
		s.reply(req, map[string]any{"type": "init_ok"})
	case "topology": // main.go:132-149: the neighbour map is replaced wholesale (:142)
		var b struct {
			Topology map[string][]string `json:"topology"`
		}
		if err := json.Unmarshal(req.Body, &b); err != nil {
			s.fail(req, errCrash, err.Error())
			return nil
		}
		s.topo = b.Topology
		for _, e := range s.pages {
			if err := e.SetTopologyMap(s.topo); err != nil {
				s.fail(req, errCrash, err.Error())
				return nil
			}
		}
		s.reply(req, map[string]any{"type": "topology_ok"})
	case "broadcast": // main.go:102-121: ack (:109), dedupe (:113), record (:117), gossip (:118)
		var b struct {
			Message *int64 `json:"message"`
		}
		if err := json.Unmarshal(req.Body, &b); err != nil || b.Message == nil {
			s.fail(req, errCrash, "message must be an integer")
			return nil
		}
		s.reply(req, map[string]any{"type": "broadcast_ok"})
		node, err := gossipgpu.NodeIndex(req.Dest)
		if err != nil {
			return err
		}
		slot, seen := s.slotOf[*b.Message]
		if !seen {
			slot = uint32(len(s.values))
			s.slotOf[*b.Message] = slot
			s.values = append(s.values, *b.Message)
			if int(slot/s.pageValues) >= len(s.pages) {
				if _, err := s.newPage(); err != nil {
					return err
				}
			}
		}
		e := s.pages[slot/s.pageValues]
		held, err := e.Read(uint64(node))
		if err != nil {
			return err
		}
		for _, h := range held {
			if h == slot%s.pageValues {
				return nil // dedupe, main.go:113
			}
		}
		if err := e.Inject(uint64(node), slot%s.pageValues); err != nil {
			return err
		}
		max := uint32(1 << 16)
		if s.topo == nil {
			max = 1 // nil Topology: marked forwarded, never sent
		}
		st, _, err := e.Step(max)
		if err != nil {
			return err
		}
		for _, r := range st {
			s.rounds++
			s.messages += r.Messages
		}
	case "read": // main.go:123-130
		node, err := gossipgpu.NodeIndex(req.Dest)
		if err != nil {
			return err
		}
		msgs := []int64{}
		for p, e := range s.pages {
			slots, err := e.Read(uint64(node))
			if err != nil {
				return err
			}
			for _, sl := range slots {
				if g := uint32(p)*s.pageValues + sl; int(g) < len(s.values) {
					msgs = append(msgs, s.values[g])
				}
			}
		}
		s.reply(req, map[string]any{"type": "read_ok", "messages": msgs})
	case "broadcast_ok": // main.go:151-153
	default:
		s.fail(req, errNotSupported, fmt.Sprintf("no handler for %q", head.Type))
	}
	return nil
}

func main() {
	page := flag.Uint("page-values", 1024, "rumor slots per engine page (1..4096)")
	flag.Parse()
	if *page < 1 || *page > 4096 { // the engine's rumor slots (gossip_create), as gossip_hip.Cluster
		fmt.Fprintln(os.Stderr, "-page-values must be in [1, 4096]")
		os.Exit(2)
	}
	s := &server{pageValues: uint32(*page), slotOf: map[int64]uint32{}, msgID: map[string]int64{},
		out: bufio.NewWriter(os.Stdout)}
	in := bufio.NewScanner(os.Stdin)
	in.Buffer(make([]byte, 1<<20), 1<<26)
	for in.Scan() {
		var req envelope
		if err := json.Unmarshal(in.Bytes(), &req); err != nil {
			fmt.Fprintln(os.Stderr, "bad json:", err)
			continue
		}
		if err := s.handle(req); err != nil {
			fmt.Fprintln(os.Stderr, "engine:", err)
			os.Exit(1)
		}
		s.out.Flush()
	}
	for _, e := range s.pages {
		e.Close()
	}
	fmt.Fprintf(os.Stderr, "gossip rounds %d, node-to-node messages %d\n", s.rounds, s.messages)
}
