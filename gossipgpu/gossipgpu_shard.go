// Per-kind steps of a sharded round (include/gossip_shard.h): for a Go host that runs the
// collectives on its own RCCL communicator instead of letting gossip_step drive them.  The
// usual multi-GPU path needs none of this (CommInitRank + Step, gossipgpu.go).
package gossipgpu

/*
#cgo CFLAGS: -I${SRCDIR}/../include
#include "gossip_shard.h"
*/
import "C"

import (
	"fmt"
	"unsafe"
)

// Exchange dense round item id flags (gossip_xd_requests).
const (
	XDNoPush uint32 = uint32(C.GOSSIP_XD_NO_PUSH)
	XDNoPull uint32 = uint32(C.GOSSIP_XD_NO_PULL)
)

// --- sharded rounds (G > 1): the host runs the collectives on its own RCCL communicator -----
// Device pointers are returned as uintptr; see include/gossip_shard.h and DESIGN.md §5 for the
// order of calls (gossip_hip/sharded.py is the same sequence in Python).

// PartialLen is the length of the stats partial vector that is all-reduced (SUM) each round.
func (e *Engine) PartialLen() uint64 { return uint64(C.gossip_partial_len(e.h)) }

// ShardedPlan: -1 / -2 need totals / the global max vector first; 0 dense, 1 sparse, 2 anti-entropy.
// total is nil or the all-reduced totals (PartialLen words; the max vector: Rumors words).
func (e *Engine) ShardedPlan(total []uint64) (int32, error) {
	if total != nil && uint64(len(total)) < e.PartialLen() {
		return 0, fmt.Errorf("gossipgpu: ShardedPlan wants %d totals", e.PartialLen())
	}
	var kind C.int32_t
	err := e.locked(func() C.int { return C.gossip_sharded_plan(e.h, u64p(total), &kind) })
	return int32(kind), err
}

// LocalTotals are the owned nodes' totals (to all-reduce before planning).
func (e *Engine) LocalTotals() ([]uint64, error) {
	out := make([]uint64, e.PartialLen())
	return out, e.locked(func() C.int { return C.gossip_local_totals(e.h, u64p(out)) })
}

// ExchangeBuffers returns the send slice and the gathered image of an all-gather (in place).
func (e *Engine) ExchangeBuffers() (send, recv uintptr, bytes uint64, err error) {
	var s, r unsafe.Pointer
	var n C.uint64_t
	err = e.locked(func() C.int { return C.gossip_exchange_buffers(e.h, &s, &r, &n) })
	return uintptr(s), uintptr(r), uint64(n), err
}

// DensePrepare enqueues the own-slice part of a dense round while the all-gather runs.
func (e *Engine) DensePrepare() error {
	return e.locked(func() C.int { return C.gossip_dense_prepare(e.h) })
}

// RoundCompute computes a dense round's S_{t+1} and returns its partial stats.
func (e *Engine) RoundCompute() ([]uint64, error) {
	out := make([]uint64, e.PartialLen())
	return out, e.locked(func() C.int { return C.gossip_round_compute(e.h, u64p(out)) })
}

// RoundCommit takes the all-reduced totals (PartialLen words) and ends the round.
func (e *Engine) RoundCommit(total []uint64) (RoundStats, error) {
	if uint64(len(total)) < e.PartialLen() {
		return RoundStats{}, fmt.Errorf("gossipgpu: RoundCommit wants %d totals", e.PartialLen())
	}
	var st C.gossip_round_stats_t
	if err := e.locked(func() C.int { return C.gossip_round_commit(e.h, u64p(total), &st) }); err != nil {
		return RoundStats{}, err
	}
	return RoundStats{Round: uint32(st.round), Converged: st.converged != 0, FullNodes: uint64(st.full_nodes),
		AliveNodes: uint64(st.alive_nodes), Messages: uint64(st.messages), StateHash: uint64(st.state_hash)}, nil
}

// SparseRare: the own rare nodes (16-B items) of a sparse round.
func (e *Engine) SparseRare() (send uintptr, count uint64, err error) {
	var s unsafe.Pointer
	var n C.uint64_t
	err = e.locked(func() C.int { return C.gossip_sparse_rare(e.h, &s, &n) })
	return uintptr(s), uint64(n), err
}

// SparseRareRecv: room for G * stride rare items.
func (e *Engine) SparseRareRecv(stride uint64) (uintptr, error) {
	var r unsafe.Pointer
	err := e.locked(func() C.int { return C.gossip_sparse_rare_recv(e.h, C.uint64_t(stride), &r) })
	return uintptr(r), err
}

// SparseScan: the pushes for other shards, grouped by owner (counts: every shard's rare count).
func (e *Engine) SparseScan(counts []uint64) (send uintptr, sendCounts []uint64, err error) {
	if len(counts) != int(e.cfg.ShardCount) {
		return 0, nil, fmt.Errorf("gossipgpu: SparseScan wants %d counts", e.cfg.ShardCount)
	}
	var s unsafe.Pointer
	sendCounts = make([]uint64, len(counts))
	err = e.locked(func() C.int { return C.gossip_sparse_scan(e.h, u64p(counts), &s, u64p(sendCounts)) })
	return uintptr(s), sendCounts, err
}

// SparseMsgRecv: room for the incoming push items.
func (e *Engine) SparseMsgRecv(items uint64) (uintptr, error) {
	var r unsafe.Pointer
	err := e.locked(func() C.int { return C.gossip_sparse_msg_recv(e.h, C.uint64_t(items), &r) })
	return uintptr(r), err
}

// SparseCommit ends a sparse round with the received pushes.
func (e *Engine) SparseCommit(items uint64) ([]uint64, error) {
	out := make([]uint64, e.PartialLen())
	return out, e.locked(func() C.int { return C.gossip_sparse_commit(e.h, C.uint64_t(items), u64p(out)) })
}

// AEItemWords: uint32 words of a request (0) or reply (1) item of sharded ANTIENTROPY.
func (e *Engine) AEItemWords(which uint32) uint32 { return uint32(C.gossip_ae_item_words(e.h, C.uint32_t(which))) }

// AELocalTarget: the max over the owned rows (all-reduce it with MAX, then AESetTarget).
func (e *Engine) AELocalTarget() ([]uint32, error) {
	out := make([]uint32, e.cfg.Rumors)
	return out, e.locked(func() C.int { return C.gossip_ae_local_target(e.h, u32p(out)) })
}

// AESetTarget installs the global max vector (Rumors words).
func (e *Engine) AESetTarget(target []uint32) error {
	if len(target) != int(e.cfg.Rumors) {
		return fmt.Errorf("gossipgpu: AESetTarget wants %d components", e.cfg.Rumors)
	}
	return e.locked(func() C.int { return C.gossip_ae_set_target(e.h, u32p(target)) })
}

// AERequests: this round's request items grouped by owner.
func (e *Engine) AERequests() (send uintptr, counts []uint64, err error) {
	var s unsafe.Pointer
	counts = make([]uint64, e.cfg.ShardCount)
	err = e.locked(func() C.int { return C.gossip_ae_requests(e.h, &s, u64p(counts)) })
	return uintptr(s), counts, err
}

// AERequestRecv: room for the incoming requests.
func (e *Engine) AERequestRecv(items uint64) (uintptr, error) {
	var r unsafe.Pointer
	err := e.locked(func() C.int { return C.gossip_ae_request_recv(e.h, C.uint64_t(items), &r) })
	return uintptr(r), err
}

// AEServe merges the received requests and returns the replies (received order).
func (e *Engine) AEServe() (uintptr, error) {
	var s unsafe.Pointer
	err := e.locked(func() C.int { return C.gossip_ae_serve(e.h, &s) })
	return uintptr(s), err
}

// AEResponseRecv: room for the replies to the own requests (request order).
func (e *Engine) AEResponseRecv() (uintptr, error) {
	var r unsafe.Pointer
	err := e.locked(func() C.int { return C.gossip_ae_response_recv(e.h, &r) })
	return uintptr(r), err
}

// AEFinish merges the replies and returns the round's partial stats.
func (e *Engine) AEFinish() ([]uint64, error) {
	out := make([]uint64, e.PartialLen())
	return out, e.locked(func() C.int { return C.gossip_ae_finish(e.h, u64p(out)) })
}

// XDClasses: with bytes > 0 this exchange round filters its edges by the peer's class: the
// driver all-gathers bytes from every rank's send slot into image (own slot in place) before
// XDRequests.  bytes == 0: nothing to gather.
func (e *Engine) XDClasses() (send, image uintptr, bytes uint64, err error) {
	var s, i unsafe.Pointer
	var n C.uint64_t
	err = e.locked(func() C.int { return C.gossip_xd_classes(e.h, &s, &i, &n) })
	return uintptr(s), uintptr(i), uint64(n), err
}

// XDRequests: the items of an exchange dense round (plan kind 3) grouped by owner: ids (uint32,
// p at its owner | XDNoPush / XDNoPull) and values (uint64), two device arrays.
func (e *Engine) XDRequests() (ids, vals uintptr, counts []uint64, err error) {
	var i, v unsafe.Pointer
	counts = make([]uint64, e.cfg.ShardCount)
	err = e.locked(func() C.int { return C.gossip_xd_requests(e.h, &i, &v, u64p(counts)) })
	return uintptr(i), uintptr(v), counts, err
}

// XDRequestRecv: room for the incoming items (ids and values).
func (e *Engine) XDRequestRecv(items uint64) (ids, vals uintptr, err error) {
	var i, v unsafe.Pointer
	err = e.locked(func() C.int { return C.gossip_xd_request_recv(e.h, C.uint64_t(items), &i, &v) })
	return uintptr(i), uintptr(v), err
}

// XDServe applies the received pushes and returns the pull replies (received order).
func (e *Engine) XDServe() (uintptr, error) {
	var s unsafe.Pointer
	err := e.locked(func() C.int { return C.gossip_xd_serve(e.h, &s) })
	return uintptr(s), err
}

// XDResponseRecv: room for the replies to the own items (send order).
func (e *Engine) XDResponseRecv() (uintptr, error) {
	var r unsafe.Pointer
	err := e.locked(func() C.int { return C.gossip_xd_response_recv(e.h, &r) })
	return uintptr(r), err
}

// XDFinish merges the replies and returns the round's partial stats.
func (e *Engine) XDFinish() ([]uint64, error) {
	out := make([]uint64, e.PartialLen())
	return out, e.locked(func() C.int { return C.gossip_xd_finish(e.h, u64p(out)) })
}

// Device-resident round values (ABI v9, gossip_*_dev): the same calls with their counts and partials
// left in engine memory (uint64 device pointers) for a device-side collective on the engine's stream.

// RoundComputeDev: the partials of a dense round (PartialLen values on the device).
func (e *Engine) RoundComputeDev() (partial uintptr, err error) {
	var p *C.uint64_t
	err = e.locked(func() C.int { return C.gossip_round_compute_dev(e.h, &p) })
	return uintptr(unsafe.Pointer(p)), err
}

// SparseRareDev: the own rare list and a device pointer to its count.
func (e *Engine) SparseRareDev() (send, count uintptr, err error) {
	var s unsafe.Pointer
	var c *C.uint64_t
	err = e.locked(func() C.int { return C.gossip_sparse_rare_dev(e.h, &s, &c) })
	return uintptr(s), uintptr(unsafe.Pointer(c)), err
}

// SparseScanDev: the pushes for other shards and a device pointer to the G per-owner counts.
func (e *Engine) SparseScanDev(counts []uint64) (send, sendCounts uintptr, err error) {
	if len(counts) != int(e.cfg.ShardCount) {
		return 0, 0, fmt.Errorf("gossipgpu: SparseScanDev wants %d counts", e.cfg.ShardCount)
	}
	var s unsafe.Pointer
	var c *C.uint64_t
	err = e.locked(func() C.int { return C.gossip_sparse_scan_dev(e.h, u64p(counts), &s, &c) })
	return uintptr(s), uintptr(unsafe.Pointer(c)), err
}

// SparseCommitDev ends a sparse round; the partials stay on the device.
func (e *Engine) SparseCommitDev(items uint64) (partial uintptr, err error) {
	var p *C.uint64_t
	err = e.locked(func() C.int { return C.gossip_sparse_commit_dev(e.h, C.uint64_t(items), &p) })
	return uintptr(unsafe.Pointer(p)), err
}

// XDRequestsDev: the items of an exchange round and a device pointer to the G per-owner counts.
func (e *Engine) XDRequestsDev() (ids, vals, counts uintptr, err error) {
	var i, v unsafe.Pointer
	var c *C.uint64_t
	err = e.locked(func() C.int { return C.gossip_xd_requests_dev(e.h, &i, &v, &c) })
	return uintptr(i), uintptr(v), uintptr(unsafe.Pointer(c)), err
}

// XDFinishDev merges the replies; the partials stay on the device.
func (e *Engine) XDFinishDev() (partial uintptr, err error) {
	var p *C.uint64_t
	err = e.locked(func() C.int { return C.gossip_xd_finish_dev(e.h, &p) })
	return uintptr(unsafe.Pointer(p)), err
}

// CCSend: the own occupancy bitmaps of a class-coded dense round (plan kind 4; [nz][full], bitsBytes
// bytes, the own slot of the gathered bitmap image) and the own mixed words (count uint64 words).
func (e *Engine) CCSend() (bits uintptr, bitsBytes uint64, vals uintptr, count uint64, err error) {
	var b, v unsafe.Pointer
	var nb, n C.uint64_t
	err = e.locked(func() C.int { return C.gossip_cc_send(e.h, &b, &nb, &v, &n) })
	return uintptr(b), uint64(nb), uintptr(v), uint64(n), err
}

// CCRecv: the gathered bitmap image (ShardCount slots of bitsBytes) and room for stride mixed
// words from every shard.
func (e *Engine) CCRecv(stride uint64) (bitsImage, vals uintptr, err error) {
	var b, v unsafe.Pointer
	err = e.locked(func() C.int { return C.gossip_cc_recv(e.h, C.uint64_t(stride), &b, &v) })
	return uintptr(b), uintptr(v), err
}

// CCExpand rebuilds the state image from the gathered bitmaps and mixed words (counts: every
// shard's count); the round then goes on with DensePrepare / RoundCompute.
func (e *Engine) CCExpand(counts []uint64) error {
	if len(counts) != int(e.cfg.ShardCount) {
		return fmt.Errorf("gossipgpu: CCExpand wants %d counts", e.cfg.ShardCount)
	}
	return e.locked(func() C.int { return C.gossip_cc_expand(e.h, u64p(counts)) })
}
