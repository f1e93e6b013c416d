// antientropy.h — version-vector anti-entropy kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gossip {

// AeArgs::flags bit (internal, above the ABI's GOSSIP_FLAG_*): the stale bits of S_t in ab are
// exact, so the binned dense round may skip the exchanges that cannot move a row
constexpr uint32_t kAeSbValid = 1u << 30;

struct AeArgs {
  uint32_t* V;             // S_t rows [N][K] (sparse rounds update them in place)
  uint32_t* Vn;            // dense rounds: S_{t+1} rows
  // alive + stale bitmaps, interleaved so one 16-B read answers both for a peer:
  // word 2w = alive bits, word 2w+1 = stale bits (row != target) of nodes 64w .. 64w+63
  const uint64_t* ab;      // before round t: alive after round t-1, stale of S_t
  uint64_t* abn;           // round t: alive after its churn; stale of S_t, then of S_{t+1}
  const uint32_t* target;  // global max vector (constant between injections)
  uint64_t* partial;
  uint64_t N;
  uint32_t K, L, k, t;
  uint32_t key0, key1, fail, rec;
  uint32_t flags;
  // sparse rounds: the scan's blocks own contiguous node ranges
  // (spc chunks of 64 nodes each) and list their edges in a segment of segcap
  uint64_t* aux;     // [0] stale nodes (stats kernels), [1] largest segment count (scan)
  uint32_t* segn;    // [nseg] edges each scan block found
  uint32_t* eid;     // [nseg][segcap][2] edge ends (n, p)
  uint32_t* erow;    // [nseg][segcap][2][K] S_t rows of the two ends
  uint32_t* claim;   // [N] epoch of the last fix-up pass that owned the node
  void* pmask;       // dense rounds: [N][k] push masks (components where V[n] > V[p_j]), L bits each
  uint32_t nseg, spc, segcap;
  uint32_t epoch;
  // binned sparse scan: the exchanges of every alive sender,
  // counting-sorted by the peer's tile (2^btl nodes) per region of 2^brs senders;
  // one block per tile then reads the tile's alive / stale bits from LDS and
  // lists the edges into segment = tile (nseg == bnt)
  uint32_t* brec;    // [bnreg][2^brs * k] records: p_local | (n - region base) << btl | stale(n) << (btl + brs)
  uint16_t* boff;    // [bnreg][bnt + 1] run starts inside each region
  uint32_t btl, bnt, brs, bnreg;
  uint32_t spb;      // blocks per segment in the gather / apply / fix kernels
  uint32_t dcap;     // binned dense rounds: in-edges sorted per LDS pass (0 = the kernel's capacity)
  // pipelined sparse rounds (engine step_ae): a word the previous round's launch_ae_gate wrote;
  // 0 = that round converged, overflowed its edge list or did not run, so this round's sparse
  // kernels return at once.  Null: always run.
  const uint32_t* gate;
  // pipelined sparse rounds, the emit's part (round 5): gate_out = this round's gate word, which the
  // emit computes from the previous round of the batch (gate_prev null: the batch's first round;
  // else *gate_prev open, its edge list did not overflow (its aux[1] <= segcap) and it did not
  // converge (its partial[0] != [1]), prev_partial being that round's slot of totals) and block 0
  // stores; zero / nzero: this round's slot, cleared by the emit's block 0 before any kernel adds
  uint32_t* gate_out;
  const uint32_t* gate_prev;
  const uint64_t* prev_partial;
  uint64_t* zero;
  uint32_t pl, nzero;
};

// binned sparse-scan geometry for N nodes, k exchanges per node
struct AeBinGeom {
  uint32_t tl, nt, rs, nreg;
};
AeBinGeom ae_bin_geom(uint64_t N, uint32_t k);
bool ae_bin_fits(const AeBinGeom& g);  // the emit's LDS tile counters cover g.nt (else the direct scan)

uint32_t ae_lanes(uint32_t K);
hipError_t launch_ae_init(uint32_t* V, uint32_t* target, uint64_t N, uint32_t K, uint32_t k0, uint32_t k1,
                          hipStream_t st);
hipError_t launch_ae_inject(uint32_t* V, uint32_t* target, uint64_t node, uint32_t K, uint32_t c, hipStream_t st);
hipError_t launch_ae_fill_alive(uint64_t* ab, uint64_t N, hipStream_t st);
// churn of round t: ab -> abn (alive bits churned, stale bits carried)
hipError_t launch_ae_churn(const AeArgs& a, hipStream_t st);
// dense round (after the churn): pull pass writes every row of Vn, push pass atomicMax into Vn
hipError_t launch_ae_round(const AeArgs& a, hipStream_t st);
// stats of (V, the alive bits of ab); write_stale also rebuilds ab's stale bits and aux[0]
hipError_t launch_ae_stats(const AeArgs& a, const uint32_t* V, uint64_t* ab, bool write_stale, hipStream_t st);
// sparse round (after the churn): scan (edges touching a stale node), gather, apply in
// place, fix-up (stale bits, hash delta into partial[3]), then stats from the bitmaps
hipError_t launch_ae_sparse(const AeArgs& a, hipStream_t st);
// the same round with the binned scan (a.brec set, a.nseg == a.bnt); its first
// pass also does the churn (no launch_ae_churn before it)
hipError_t launch_ae_sparse_binned(const AeArgs& a, hipStream_t st);
hipError_t launch_ae_sparse_stats(const AeArgs& a, hipStream_t st);
// binned dense round: geometry of its 2^14-node tiles (the sparse scan's
// sender regions), whether the kernels' LDS tables cover it, and the round itself: the
// emit (churn fused, records into a.brec, run starts into a.boff with a.btl / a.bnt of
// this geometry), then one block per tile writes every row of Vn, the stale bits of abn
// and the round's stats (no launch_ae_stats after it); aux[1] != 0: a chunk's in-edges
// overflowed the LDS list, rerun the round with launch_ae_round
AeBinGeom ae_dense_geom(uint64_t N, uint32_t k);
bool ae_dense_fits(const AeBinGeom& g, uint64_t N, uint32_t k, uint32_t K);
hipError_t launch_ae_dense_binned(const AeArgs& a, hipStream_t st);

}  // namespace gossip
