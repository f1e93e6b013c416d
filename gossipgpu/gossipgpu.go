// Package gossipgpu binds the MI355X gossip-round engine (libgossip_hip.so, the C ABI of
// include/gossip.h, ABI v10) for Go hosts such as 0xSherlokMo/gossip-protocol's main.go.
//
// The reference floods each value once to its topology neighbours with blocking SyncRPCs
// ((*NodeState).Gossip, main.go:65-89), one process per node.  Here one Engine holds every
// node's state in HBM and runs the dissemination as synchronous rounds:
//
//	topology handler  (main.go:132-149)  -> SetTopology / SetTopologyMap
//	broadcast handler (main.go:102-121)  -> Inject, then Step (replaces State.Gossip, :118)
//	read handler      (main.go:123-130)  -> Read
//
// Several GPUs (DESIGN.md §5.5): one Engine per GPU with ShardRank / ShardCount set; rank 0
// calls CommUniqueID, every rank gets the bytes and calls CommInitRank, then Step on every
// rank runs the sharded rounds over the engines' own RCCL communicators.  Or one process
// holds all shards: NewGroup + Group.Step.
//
// Errors are *Error values carrying the gossip_status code and gossip_last_error().  One
// Engine serializes its calls with a mutex (the library is not thread-safe per engine; the
// reference guards MessageKeeper with sync.RWMutex, main.go:25).  Host slices are read only
// for the duration of a call and never retained (the cgo pointer rules).
//
// Build: make -C gossip-protocol_amd (hipcc, gfx950); then go build ./... here.  This image
// has no Go toolchain, so the package is checked by tests/test_go_binding.py (every call and
// config field against include/gossip.h), not compiled.
package gossipgpu

/*
#cgo CFLAGS: -I${SRCDIR}/../include
#cgo LDFLAGS: -L${SRCDIR}/../gossip-protocol_amd/gossip_hip -lgossip_hip -Wl,-rpath,${SRCDIR}/../gossip-protocol_amd/gossip_hip
#include <stdlib.h>
#include "gossip.h"
*/
import "C"

import (
	"bytes"
	"fmt"
	"sort"
	"strconv"
	"sync"
	"unsafe"
)

// ABIVersion is the gossip.h version this binding is written against.
const ABIVersion = 10

// Mode is a dissemination rule (DESIGN.md §2).
type Mode uint32

const (
	Flood       Mode = Mode(C.GOSSIP_MODE_FLOOD) // the reference's own algorithm, main.go:65-89
	Push        Mode = Mode(C.GOSSIP_MODE_PUSH)
	Pull        Mode = Mode(C.GOSSIP_MODE_PULL)
	PushPull    Mode = Mode(C.GOSSIP_MODE_PUSHPULL)
	AntiEntropy Mode = Mode(C.GOSSIP_MODE_ANTIENTROPY)
)

// Flags select optional outputs and A/B round paths (results never change).
type Flags uint32

const (
	FlagHash         Flags = Flags(C.GOSSIP_FLAG_HASH)
	FlagTiming       Flags = Flags(C.GOSSIP_FLAG_TIMING)
	FlagDirect       Flags = Flags(C.GOSSIP_FLAG_DIRECT)
	FlagDense        Flags = Flags(C.GOSSIP_FLAG_DENSE)
	FlagShardDirect  Flags = Flags(C.GOSSIP_FLAG_SHARD_DIRECT)
	FlagAEDirectScan Flags = Flags(C.GOSSIP_FLAG_AE_DIRECT_SCAN)
)

// Config mirrors gossip_config_t.  Probabilities are thresholds x / 2^32 (Threshold).
type Config struct {
	Nodes        uint64 // N, 2 <= N < 2^32
	Rumors       uint32 // R rumor slots (ANTIENTROPY: K version components)
	Mode         Mode
	Fanout       uint32 // Philox peers per node per round (random modes, ANTIENTROPY)
	Flags        Flags
	Seed         uint64
	Device       int32 // HIP device ordinal, -1 = current
	ShardRank    uint32
	ShardCount   uint32 // 0 or 1: one engine holds every node
	ChurnFail    uint32 // ANTIENTROPY churn
	ChurnRecover uint32
	EdgeLoss     uint32 // fault model (DESIGN.md §2.8)
	Partitions   uint32
	StallRounds  uint32 // the reference's expired-context stall (DESIGN.md §2.9), 0 = off
}

// Threshold converts a probability into the x / 2^32 threshold of the config fields.
func Threshold(p float64) uint32 {
	if p <= 0 {
		return 0
	}
	if p >= 1 {
		return ^uint32(0)
	}
	return uint32(p * 4294967296.0)
}

// Error is a failed call: the gossip_status code and the engine's message.
type Error struct {
	Code int
	Msg  string
}

var statusNames = map[int]string{
	int(C.GOSSIP_EINVAL): "EINVAL", int(C.GOSSIP_EHIP): "EHIP", int(C.GOSSIP_ENOMEM): "ENOMEM",
	int(C.GOSSIP_ESTATE): "ESTATE", int(C.GOSSIP_ENODEV): "ENODEV", int(C.GOSSIP_ENOTSUP): "ENOTSUP",
	int(C.GOSSIP_ERCCL): "ERCCL",
}

func (e *Error) Error() string { return fmt.Sprintf("gossip %s: %s", statusNames[e.Code], e.Msg) }

// RoundStats mirrors gossip_round_stats_t: the state S_{t+1} that round t produced.
type RoundStats struct {
	Round      uint32
	Converged  bool
	FullNodes  uint64
	AliveNodes uint64
	Messages   uint64 // FLOOD: broadcast RPCs sent; ANTIENTROPY: exchanges between alive nodes
	StateHash  uint64 // FlagHash only
}

// Engine is one gossip_engine_t.
type Engine struct {
	mu  sync.Mutex
	h   *C.gossip_engine_t
	cfg Config
}

func (e *Engine) fail(rc C.int) error {
	return &Error{Code: int(rc), Msg: C.GoString(C.gossip_last_error(e.h))}
}

// New creates an engine (NewState / NewMessageKeeper, main.go:28-33, 91-97).  It fails with
// ENODEV without a gfx950 device: the library has no CPU fallback.
func New(cfg Config) (*Engine, error) {
	if v := uint32(C.gossip_abi_version()); v != ABIVersion {
		return nil, fmt.Errorf("gossipgpu: libgossip_hip ABI %d, binding written for %d", v, ABIVersion)
	}
	c := cConfig(cfg)
	var h *C.gossip_engine_t
	if rc := C.gossip_create(&c, &h); rc != 0 {
		return nil, &Error{Code: int(rc), Msg: C.GoString(C.gossip_last_error(nil))}
	}
	return &Engine{h: h, cfg: cfg}, nil
}

func cConfig(cfg Config) C.gossip_config_t {
	return C.gossip_config_t{
		n_nodes: C.uint64_t(cfg.Nodes), n_rumors: C.uint32_t(cfg.Rumors), mode: C.uint32_t(cfg.Mode),
		fanout: C.uint32_t(cfg.Fanout), flags: C.uint32_t(cfg.Flags), seed: C.uint64_t(cfg.Seed),
		device: C.int32_t(cfg.Device), shard_rank: C.uint32_t(cfg.ShardRank), shard_count: C.uint32_t(cfg.ShardCount),
		churn_fail: C.uint32_t(cfg.ChurnFail), churn_recover: C.uint32_t(cfg.ChurnRecover),
		edge_loss: C.uint32_t(cfg.EdgeLoss), partitions: C.uint32_t(cfg.Partitions),
		stall_rounds: C.uint32_t(cfg.StallRounds),
	}
}

// Close releases every device buffer.
func (e *Engine) Close() {
	e.mu.Lock()
	defer e.mu.Unlock()
	if e.h != nil {
		C.gossip_destroy(e.h)
		e.h = nil
	}
}

func u32p(s []uint32) *C.uint32_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint32_t)(unsafe.Pointer(&s[0]))
}

func u64p(s []uint64) *C.uint64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint64_t)(unsafe.Pointer(&s[0]))
}

// SetTopology installs Topology[u] = col[rowPtr[u]:rowPtr[u+1]] (the topology handler,
// main.go:132-149, State.Topology = body.Topology at :142).  Rows are sets.
func (e *Engine) SetTopology(rowPtr, col []uint32) error {
	e.mu.Lock()
	defer e.mu.Unlock()
	if len(rowPtr) == 0 {
		return &Error{Code: int(C.GOSSIP_EINVAL), Msg: "empty row_ptr"}
	}
	rc := C.gossip_set_topology_csr(e.h, u32p(rowPtr), u32p(col), C.uint64_t(len(rowPtr)-1), C.uint64_t(len(col)))
	if rc != 0 {
		return e.fail(rc)
	}
	return nil
}

// NodeIndex maps a Maelstrom node id "n<k>" to k.
func NodeIndex(id string) (uint32, error) {
	if len(id) < 2 || id[0] != 'n' {
		return 0, fmt.Errorf("gossipgpu: node id %q is not n<k>", id)
	}
	k, err := strconv.ParseUint(id[1:], 10, 32)
	return uint32(k), err
}

// SetTopologyMap installs the body of a Maelstrom topology message (map node id -> neighbour ids).
func (e *Engine) SetTopologyMap(topo map[string][]string) error {
	rows := make([][]uint32, e.cfg.Nodes)
	for src, nbrs := range topo {
		u, err := NodeIndex(src)
		if err != nil {
			return err
		}
		if uint64(u) >= e.cfg.Nodes {
			return fmt.Errorf("gossipgpu: node %s outside the cluster", src)
		}
		for _, d := range nbrs {
			v, err := NodeIndex(d)
			if err != nil {
				return err
			}
			rows[u] = append(rows[u], v)
		}
		sort.Slice(rows[u], func(a, b int) bool { return rows[u][a] < rows[u][b] })
	}
	rowPtr := make([]uint32, e.cfg.Nodes+1)
	var col []uint32
	for u, r := range rows {
		col = append(col, r...)
		rowPtr[u+1] = uint32(len(col))
	}
	return e.SetTopology(rowPtr, col)
}

func (e *Engine) call(rc C.int) error {
	if rc != 0 {
		return e.fail(rc)
	}
	return nil
}

// Reset clears every rumor bit (and versions / alive flags) and the round index.
func (e *Engine) Reset() error {
	e.mu.Lock()
	defer e.mu.Unlock()
	return e.call(C.gossip_reset(e.h))
}

// Inject is a client broadcast of rumor slot `slot` at `node` (main.go:102-117; a repeat is
// the dedupe of :113).  ANTIENTROPY: a local write of component `slot`.
func (e *Engine) Inject(node uint64, slot uint32) error {
	e.mu.Lock()
	defer e.mu.Unlock()
	return e.call(C.gossip_inject(e.h, C.uint64_t(node), C.uint32_t(slot)))
}

// InjectRandom puts every rumor at its Philox origin (ANTIENTROPY: random initial versions).
func (e *Engine) InjectRandom() error {
	e.mu.Lock()
	defer e.mu.Unlock()
	return e.call(C.gossip_inject_random(e.h))
}

// SetFaults changes the fault model between steps (e.g. heal a partition with parts = 0).
func (e *Engine) SetFaults(edgeLoss, partitions uint32) error {
	e.mu.Lock()
	defer e.mu.Unlock()
	return e.call(C.gossip_set_faults(e.h, C.uint32_t(edgeLoss), C.uint32_t(partitions)))
}

// SetParam sets a tuning / path-selection knob (gossip_set_param); results never change.
func (e *Engine) SetParam(name string, value float64) error {
	e.mu.Lock()
	defer e.mu.Unlock()
	cs := C.CString(name)
	defer C.free(unsafe.Pointer(cs))
	return e.call(C.gossip_set_param(e.h, cs, C.double(value)))
}

// SetStream binds a hipStream_t (nil: the null stream).
func (e *Engine) SetStream(stream unsafe.Pointer) error {
	e.mu.Lock()
	defer e.mu.Unlock()
	return e.call(C.gossip_set_stream(e.h, stream))
}

// Step runs rounds until every node holds every rumor (FLOOD also: until a round sends
// nothing) or maxRounds ran.  It replaces State.Gossip (main.go:118).  With ShardCount > 1
// the engine needs CommInitRank first and every rank calls Step with the same maxRounds;
// the stats are global.  infected[t][r] = nodes holding rumor r after round t.
func (e *Engine) Step(maxRounds uint32) ([]RoundStats, [][]uint64, error) {
	e.mu.Lock()
	defer e.mu.Unlock()
	if maxRounds == 0 {
		return nil, nil, nil
	}
	st := make([]C.gossip_round_stats_t, maxRounds)
	R := uint64(e.cfg.Rumors)
	inf := make([]uint64, uint64(maxRounds)*R)
	var done C.uint32_t
	if rc := C.gossip_step(e.h, C.uint32_t(maxRounds), &st[0], u64p(inf), &done); rc != 0 {
		return nil, nil, e.fail(rc)
	}
	out, rows := convertStats(st, inf, int(done), R)
	return out, rows, nil
}

func convertStats(st []C.gossip_round_stats_t, inf []uint64, n int, R uint64) ([]RoundStats, [][]uint64) {
	out := make([]RoundStats, n)
	rows := make([][]uint64, n)
	for i := 0; i < n; i++ {
		out[i] = RoundStats{Round: uint32(st[i].round), Converged: st[i].converged != 0,
			FullNodes: uint64(st[i].full_nodes), AliveNodes: uint64(st[i].alive_nodes),
			Messages: uint64(st[i].messages), StateHash: uint64(st[i].state_hash)}
		rows[i] = inf[uint64(i)*R : uint64(i+1)*R]
	}
	return out, rows
}

// UniqueIDBytes is the size of an RCCL unique id (gossip_comm_unique_id).
const UniqueIDBytes = int(C.GOSSIP_UNIQUE_ID_BYTES)

// CommUniqueID makes the RCCL unique id (rank 0); hand it to every rank by any channel.
func CommUniqueID() ([]byte, error) {
	buf := make([]byte, UniqueIDBytes)
	if rc := C.gossip_comm_unique_id((*C.uint8_t)(unsafe.Pointer(&buf[0]))); rc != 0 {
		return nil, &Error{Code: int(rc), Msg: C.GoString(C.gossip_last_error(nil))}
	}
	return buf, nil
}

// CommInitRank joins this engine (ShardRank of ShardCount) to the RCCL communicator of id;
// Step then runs sharded rounds (DESIGN.md §5.5).  Every rank calls it.
func (e *Engine) CommInitRank(id []byte) error {
	if len(id) != UniqueIDBytes {
		return fmt.Errorf("gossipgpu: CommInitRank wants %d bytes", UniqueIDBytes)
	}
	return e.locked(func() C.int { return C.gossip_comm_init_rank(e.h, (*C.uint8_t)(unsafe.Pointer(&id[0]))) })
}

// Transport of a Group.
const (
	TransportAuto int32 = 0 // RCCL when every shard has its own device, else device copies
	TransportRCCL int32 = 1
	TransportCopy int32 = 2
)

// Group is every shard of one run in this process (gossip_group_*): one engine per shard,
// the rounds driven by the library.
type Group struct {
	mu     sync.Mutex
	g      *C.gossip_group_t
	cfg    Config
	shards []*Engine
}

// NewGroup creates shards engines (devices: one ordinal per shard, or nil = cfg.Device).
func NewGroup(cfg Config, shards uint32, devices []int32, transport int32) (*Group, error) {
	if devices != nil && len(devices) != int(shards) {
		return nil, fmt.Errorf("gossipgpu: NewGroup wants %d devices", shards)
	}
	c := cConfig(cfg)
	var devp *C.int32_t
	if devices != nil {
		devp = (*C.int32_t)(unsafe.Pointer(&devices[0]))
	}
	var g *C.gossip_group_t
	if rc := C.gossip_group_create(&c, C.uint32_t(shards), devp, C.int32_t(transport), &g); rc != 0 {
		return nil, &Error{Code: int(rc), Msg: C.GoString(C.gossip_group_last_error(nil))}
	}
	grp := &Group{g: g, cfg: cfg}
	for r := uint32(0); r < shards; r++ {
		sc := cfg
		sc.ShardRank, sc.ShardCount = r, shards
		grp.shards = append(grp.shards, &Engine{h: C.gossip_group_engine(g, C.uint32_t(r)), cfg: sc})
	}
	return grp, nil
}

// Transport is the group's transport: TransportRCCL or TransportCopy (0 for one shard).
func (g *Group) Transport() int32 { return int32(C.gossip_group_transport(g.g)) }

// Shard is the engine of shard rank (owned by the group: do not Close it).
func (g *Group) Shard(rank uint32) *Engine { return g.shards[rank] }

// Step runs rounds over every shard (as Engine.Step).
func (g *Group) Step(maxRounds uint32) ([]RoundStats, [][]uint64, error) {
	g.mu.Lock()
	defer g.mu.Unlock()
	if maxRounds == 0 {
		return nil, nil, nil
	}
	for _, e := range g.shards { // no shard call may run while the group steps
		e.mu.Lock()
		defer e.mu.Unlock()
	}
	st := make([]C.gossip_round_stats_t, maxRounds)
	R := uint64(g.cfg.Rumors)
	inf := make([]uint64, uint64(maxRounds)*R)
	var done C.uint32_t
	if rc := C.gossip_group_step(g.g, C.uint32_t(maxRounds), &st[0], u64p(inf), &done); rc != 0 {
		return nil, nil, &Error{Code: int(rc), Msg: C.GoString(C.gossip_group_last_error(g.g))}
	}
	out, rows := convertStats(st, inf, int(done), R)
	return out, rows, nil
}

// Close releases every shard.
func (g *Group) Close() {
	g.mu.Lock()
	defer g.mu.Unlock()
	if g.g != nil {
		for _, e := range g.shards {
			e.mu.Lock()
			e.h = nil
			e.mu.Unlock()
		}
		C.gossip_group_destroy(g.g)
		g.g = nil
	}
}

// ReadBitset is the word form of the read handler (main.go:123-130).
func (e *Engine) ReadBitset(node uint64) ([]uint64, error) {
	e.mu.Lock()
	defer e.mu.Unlock()
	w := (e.cfg.Rumors + 63) / 64
	out := make([]uint64, w)
	if rc := C.gossip_read_bitset(e.h, C.uint64_t(node), u64p(out), C.uint32_t(w)); rc != 0 {
		return nil, e.fail(rc)
	}
	return out, nil
}

// Read returns the rumor slots node holds (the read handler, main.go:123-130).
func (e *Engine) Read(node uint64) ([]uint32, error) {
	words, err := e.ReadBitset(node)
	if err != nil {
		return nil, err
	}
	var slots []uint32
	for r := uint32(0); r < e.cfg.Rumors; r++ {
		if (words[r/64]>>(r%64))&1 == 1 {
			slots = append(slots, r)
		}
	}
	return slots, nil
}

// ReadShard returns the owned shard's words, out[w*n + i] for owned node lo + i.
func (e *Engine) ReadShard() ([]uint64, error) {
	lo, hi := e.ShardRange()
	e.mu.Lock()
	defer e.mu.Unlock()
	out := make([]uint64, uint64((e.cfg.Rumors+63)/64)*(hi-lo))
	if rc := C.gossip_read_shard(e.h, u64p(out), C.uint64_t(len(out))); rc != 0 {
		return nil, e.fail(rc)
	}
	return out, nil
}

// ReadVersions returns one node's K versions and its alive flag (ANTIENTROPY).
func (e *Engine) ReadVersions(node uint64) ([]uint32, bool, error) {
	e.mu.Lock()
	defer e.mu.Unlock()
	out := make([]uint32, e.cfg.Rumors)
	var alive C.uint32_t
	if rc := C.gossip_read_versions(e.h, C.uint64_t(node), u32p(out), C.uint32_t(len(out)), &alive); rc != 0 {
		return nil, false, e.fail(rc)
	}
	return out, alive != 0, nil
}

// ReadRows returns every owned row (ANTIENTROPY), out[i*K + c].
func (e *Engine) ReadRows() ([]uint32, error) {
	lo, hi := e.ShardRange()
	e.mu.Lock()
	defer e.mu.Unlock()
	out := make([]uint32, (hi-lo)*uint64(e.cfg.Rumors))
	if rc := C.gossip_read_rows(e.h, u32p(out), C.uint64_t(len(out))); rc != 0 {
		return nil, e.fail(rc)
	}
	return out, nil
}

// StateHash is the order-independent state hash (DESIGN.md §2.5).
func (e *Engine) StateHash() (uint64, error) {
	e.mu.Lock()
	defer e.mu.Unlock()
	var h C.uint64_t
	if rc := C.gossip_state_hash(e.h, &h); rc != 0 {
		return 0, e.fail(rc)
	}
	return uint64(h), nil
}

// ShardRange is the owned node range [lo, hi).
func (e *Engine) ShardRange() (lo, hi uint64) {
	var l, h C.uint64_t
	C.gossip_shard_range(e.h, &l, &h)
	return uint64(l), uint64(h)
}

// RoundIndex is t, the rounds run since the last reset.
func (e *Engine) RoundIndex() uint32 { return uint32(C.gossip_round_index(e.h)) }

// KernelTime returns a FlagTiming timer's accumulated device ms and launch count.
func (e *Engine) KernelTime(which uint32) (float64, uint64, error) {
	var ms C.double
	var n C.uint64_t
	if rc := C.gossip_kernel_time(e.h, C.uint32_t(which), &ms, &n); rc != 0 {
		return 0, 0, e.fail(rc)
	}
	return float64(ms), uint64(n), nil
}

// ResetTiming clears the FlagTiming timers.
func (e *Engine) ResetTiming() error { return e.call(C.gossip_reset_timing(e.h)) }

// RoundWall returns, for library-driven sharded rounds of class cls (0 dense, 1 sparse,
// 2 ANTIENTROPY), the whole rounds' ms (collectives included; FlagTiming), the rounds run and
// the bytes this shard put on its links (gossip_round_wall).
func (e *Engine) RoundWall(cls uint32) (float64, uint64, uint64, error) {
	var ms C.double
	var n, lb C.uint64_t
	if rc := C.gossip_round_wall(e.h, C.uint32_t(cls), &ms, &n, &lb); rc != 0 {
		return 0, 0, 0, e.fail(rc)
	}
	return float64(ms), uint64(n), uint64(lb), nil
}

// PlanModel returns the planner's model of the sharded rounds it planned (gossip_plan_model):
// modelled per-rank ms and their link part since ResetTiming, the rounds covered, and the current
// run's plan string (S sparse, X exchange, C class-coded, D state all-gather).
func (e *Engine) PlanModel() (float64, float64, uint64, string, error) {
	var ms, link C.double
	var n C.uint64_t
	buf := make([]byte, 256)
	if rc := C.gossip_plan_model(e.h, &ms, &link, &n, (*C.char)(unsafe.Pointer(&buf[0])), C.uint32_t(len(buf))); rc != 0 {
		return 0, 0, 0, "", e.fail(rc)
	}
	plan := string(buf[:bytes.IndexByte(buf, 0)])
	return float64(ms), float64(link), uint64(n), plan, nil
}

// PhiloxDevice runs Philox4x32-10 on the device for known-answer tests (ctr: 4 words per counter).
func (e *Engine) PhiloxDevice(ctr []uint32, key [2]uint32) ([]uint32, error) {
	e.mu.Lock()
	defer e.mu.Unlock()
	out := make([]uint32, len(ctr))
	k := []uint32{key[0], key[1]}
	if rc := C.gossip_philox_device(e.h, u32p(ctr), u32p(k), u32p(out), C.uint32_t(len(ctr)/4)); rc != 0 {
		return nil, e.fail(rc)
	}
	return out, nil
}

// Peer is p_j(node, round) exactly as the kernels draw it.
func Peer(seed, nodes uint64, node, round, j uint32) uint32 {
	return uint32(C.gossip_peer(C.uint64_t(seed), C.uint64_t(nodes), C.uint32_t(node), C.uint32_t(round), C.uint32_t(j)))
}

// locked runs one cgo call under e.mu (one engine is not thread-safe, include/gossip.h).
func (e *Engine) locked(f func() C.int) error {
	e.mu.Lock()
	defer e.mu.Unlock()
	return e.call(f())
}
