// engine.hip — the C ABI of include/gossip.h over the HIP round kernels.
//
// Replaces the reference's per-process NodeState/MessageKeeper (main.go:22-63)
// and the recursive flood of (*NodeState).Gossip (main.go:65-89) with one
// engine object that holds every node's rumor words in HBM and advances all of
// them one synchronous round per gossip_step iteration.  HIP only: there is no
// CPU fallback; without a gfx950 device gossip_create fails with ENODEV.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <string>
#include <vector>

#include "../../include/gossip_shard.h"
#include "ae_sharded.h"
#include "antientropy.h"
#include "binned.h"
#include "frontier.h"
#include "sharded.h"
#include "round.h"

#include <cmath>
#include <immintrin.h>
#include "kernels.h"
#include "multi.h"
#include "philox.h"

using namespace gossip;

namespace {

thread_local std::string g_create_error;

// 0 = round kernel (binned engines: the whole step), 1 = stats kernel, 2 = ANTIENTROPY sparse round
// kernels, 3 = dense rounds of a binned engine (emit..apply, per round), 4 = its sparse rounds
constexpr int kTimers = 6;
constexpr uint32_t kRing = 8;

}  // namespace

struct gossip_engine {
  gossip_config_t cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  gossip::Transport* tr = nullptr;  // the collectives of gossip_step (G > 1), owned (gossip_comm_init_rank)
  // true only while the library itself drives the rounds (sharded_step inside gossip_step /
  // gossip_group_step: DrivenScope): its collectives run on the engine's own stream (RCCL) or
  // drain it first (copies), so a buffer handed to them needs no stream sync.  A host that runs
  // its own collectives through the per-kind calls always gets the publishing sync.
  bool driven = false;
  // gossip_set_param "ordered_collectives": the host's collectives run on streams ordered after
  // the engine's own (torch.distributed bound to the stream the engine launches on, as
  // gossip_hip.sharded binds it), so a buffer handed out needs no publishing sync either
  bool ordered = false;
  // gossip_set_param "rccl_dev_collectives": the RCCL transport's device-value collectives
  // (counts and partials read by RCCL from engine memory).  Off by default until they have run
  // on a box with two or more GPUs; off, RCCL takes the base forms (read_dev + host collectives).
  bool rccl_dev = false;
  // gossip_round_wall: whole library-driven sharded rounds by class (dense / sparse / ANTIENTROPY)
  double wall_ms[3] = {};
  uint64_t wall_n[3] = {}, wall_link[3] = {};
  hipEvent_t wall_ev[2] = {};

  uint64_t N = 0, Nl = 0, lo = 0, hi = 0, nown = 0;
  uint32_t R = 0, W = 0, k = 0, mode = 0, G = 1, rank = 0;
  uint32_t t = 0;
  uint32_t key0 = 0, key1 = 0;
  Faults fa{};  // lost edges

  // Random modes: two gathered images [G][W][Nl]; S_t is this rank's slice of
  // img[cur], S_{t+1} its slice of img[cur^1], so the all-gather runs in place.
  // FLOOD: S/Snext/Sprev/skip are shard-sized and the frontier F is the slice of imgF.
  uint64_t* img[2] = {nullptr, nullptr};
  int cur = 0;
  uint64_t* imgF = nullptr;
  uint64_t* S = nullptr;      // S_t, own shard [W][Nl]
  uint64_t* Snext = nullptr;  // S_{t+1}
  uint64_t* Sprev = nullptr;  // FLOOD S_{t-1}
  uint64_t* skip = nullptr;   // FLOOD sender-skip masks
  uint64_t* F = nullptr;      // FLOOD frontier (exchange send slice)
  uint64_t* partial_d = nullptr;
  uint64_t* partial_h = nullptr;  // pinned
  uint64_t* scratch_d = nullptr;  // 8 B
  uint32_t *orow = nullptr, *ocol = nullptr, *irow = nullptr, *icol = nullptr;
  bool has_topo = false;
  // stall mode, random modes: streak per node, all N nodes on every shard
  uint8_t* stall_d = nullptr;
  // FLOOD with faults, one shard: per out-edge pending values and first senders
  bool flood_edges = false;
  FloodWalks fw{nullptr, nullptr, nullptr, 0u};  // FLOOD with faults: the walks
  // ANTIENTROPY: rows V[n*K + c], alive bytes, global max vector
  uint32_t *V = nullptr, *Vn = nullptr, *target = nullptr;
  uint64_t *alive = nullptr, *alive_n = nullptr;  // [chunks][2]: alive bits, stale bits (AeArgs::ab)
  // ANTIENTROPY sparse rounds: stale bitmap of V, edge list + row snapshots,
  // fix-up claims; aux = [0] stale nodes [1] listed edges (device) / ae_aux_h (pinned host copy)
  // (one-engine ANTIENTROPY: aux is the two words after partial_d / partial_h, so one copy and
  // one memset per round move both)
  uint64_t *ae_aux = nullptr, *ae_aux_h = nullptr;
  bool ae_aux_alias = false;
  // one-engine ANTIENTROPY: gossip_reset's zeroing of V is pending (set_dev does it before any other
  // call; gossip_inject_random, which writes every row, drops it: a 4 GiB memset at configs[4])
  bool ae_v_zero = false;
  uint32_t *ae_eid = nullptr, *ae_erow = nullptr, *ae_claim = nullptr, *ae_segn = nullptr;
  void* ae_pmask = nullptr;  // dense rounds: [N][k] push masks
  uint32_t ae_nseg = 1, ae_spc = 1, ae_segcap = 1;
  bool ae_bin = false;  // binned sparse scan (AeArgs::brec)
  AeBinGeom ae_bg{};
  uint32_t* ae_brec = nullptr;
  uint16_t* ae_boff = nullptr;
  // binned dense rounds: run starts per region over 2^14-node tiles;
  // ae_dbin = the engine's geometry fits, ae_dbin_on = gossip_set_param "ae_dense_bin"
  bool ae_dbin = false, ae_dbin_on = true;
  uint32_t ae_dcap = 0;  // gossip_set_param "ae_dense_cap" (tests: ranges, overflow fallback)
  bool ae_dfilt = true;  // "ae_dense_filter": binned dense rounds skip exchanges that move no row (kAeSbValid)
  AeBinGeom ae_dg{};
  uint16_t* ae_dboff = nullptr;
  uint64_t ae_dense_fallbacks = 0;
  uint64_t ae_cap = 0, ae_hash = 0, ae_stale = 0, ae_alive = 0, ae_full = 0;
  uint32_t ae_epoch = 0;
  int ae_force = -1;             // param "ae_sparse": -1 auto, 0 never, 1 whenever the bitmap is valid
  bool ae_sb_valid = false;      // the stale bits of alive, ae_hash and ae_stale describe V
  bool ae_sparse_last = false;   // the last round ran in place (V not rotated)
  uint64_t ae_sparse_rounds = 0, ae_overflows = 0;
  // pipelined sparse rounds (step_ae): up to ae_ahead enqueued at once, each gated on device by its
  // predecessor; per round a slot of totals + aux and a gate word
  uint32_t ae_ahead = 8;
  bool ae_dense_next = false;    // the next round runs dense (a pipelined sparse round overflowed)
  uint64_t *ae_slot_d = nullptr, *ae_slot_h = nullptr;
  uint32_t* ae_gate_d = nullptr;
  // sharded ANTIENTROPY (G > 1): V/Vn = own rows [Nl][K], aex_img = every
  // shard's {alive, stale} word pairs (the all-gather image, ae_sharded.h AexArgs::img)
  bool aex = false;
  bool aex_target_ok = false;
  uint32_t aex_rw = 0, aex_pw = 0;
  uint64_t *aex_img = nullptr, *aex_cnt = nullptr, *aex_boff = nullptr, *aex_cnt_h = nullptr;
  uint64_t aex_churned = ~0ull;  // the round whose churn the own alive words hold
  uint32_t *aex_bcnt = nullptr, *aex_req = nullptr, *aex_loc = nullptr, *aex_in = nullptr, *aex_resp_out = nullptr,
           *aex_resp_in = nullptr, *aex_tmp = nullptr;
  uint64_t aex_req_cap = 0, aex_in_cap = 0, aex_out_cap = 0, aex_nin = 0, aex_nreq = 0, aex_nloc = 0;
  // Vn seeding (launch_aex_seed_next): after a completed round Vn holds S_{t-1} and aex_dirty marks the
  // rows that round raised, so the next round copies only those; any direct write (reset, inject) voids it
  uint64_t* aex_dirty = nullptr;  // [ceil(Nl / 64)]
  uint8_t* aex_verdict = nullptr;  // [nown] the count pass's listed exchanges per own node
  bool aex_patch_ok = false, aex_round_done = false;
  bool aex_track = false;  // this round marks the rows it raises (few items: ae_request_recv decides)
  // incremental stats (launch_aex_finish inc): the own stale words and hash part of S_t are exact
  bool aex_inc_ok = false;
  uint64_t aex_hash_own = 0;  // this shard's part of the state hash of the last committed round
  // binned (LDS) pipeline for W == 1 random modes on one shard
  bool binned = false;
  BinGeom bg{};
  BinBufs bb{};
  uint32_t* bb_dyn = nullptr;  // the tile queues (gossip_set_param "tile_queues" 0 clears bb.dyn)
  void* bin_mem = nullptr;
  // placement of the record slab (place_bins): the dense round's time depends on where the slab
  // lands (4.98-5.48 ms at 2^27 across fresh allocations in one process, profiles/r05_pl/r05_pl4/,
  // r05_pl6/); before the first round place_tries allocations are timed on a zero-state trial round
  // and the fastest is kept (param place_tries; 1: the first allocation; 16 vs 8 at 2^27:
  // 5.09 / 5.10 / 5.08 against 5.21 / 5.09 / 5.09 ms, profiles/r05_pl/r05_pl9/)
  uint32_t place_tries = 12;
  bool placed = false;
  bool ae_placed = false;  // one-engine ANTIENTROPY: rows and records placed (ae_place)
  bool sb_placed = false;  // sharded: the state all-gather rounds' slab placed (place_sb)
  // frontier (sparse-round) path, on top of the binned one
  bool frontier = false;
  FrontierBufs fb{};
  void* fr_mem = nullptr;
  bool fr_valid = false;          // partial_d holds the totals of S and the bitmaps are exact
  double sparse_frac = 1.0 / 16;  // rare fraction at or below which a round runs sparse (sparse_frac_of)
  bool sparse_frac_set = false;   // set by gossip_set_param (else the sharded defaults apply)
  double filter_frac = 0.3;       // dense rounds filter edges by the peer's class above this empty / full fraction
  bool filter_frac_set = false;   // else off past 2^25 nodes (filter_frac_of)
  double xd_filter_frac = 0.6;    // exchange rounds likewise (their probe hits a G-shard class image: G = 8 sweep)
  double alld_frac = 1.0 / 128;   // sparse rounds with k * rare >= alld_frac * N commit every group's D (sweep: profiles/r05_ad/)
  bool sparse_direct = true;      // ... and with an empty majority take the pushes into empty peers in S (kSparseDirect)
  // sparse rounds take the binned scan (frontier.hip K1a / K1b) once this share of peers would hit
  // the LDS summary (param bin_scan_frac)
  double bscan_frac = 0.6;
  double mid_frac = 0.5;          // sparse rounds test peers in the mid-level summary once this share hits the LDS one
  // pipelined rounds (binned engines): the host picks each round's path from the
  // totals it has read, predicted forward over the rounds still in flight, and
  // stays up to `ahead` rounds in front
  uint64_t* ring_h = nullptr;  // [kRing][part_len + 1] host-mapped totals + sequence word per round
  uint64_t* ring_d = nullptr;
  uint64_t seq = 0;
  uint32_t ahead = 2;
  // sharded sparse rounds (G > 1, W == 1 random modes; sharded.h):
  // lf = frontier buffers over the owned nodes, sb = rare lists, global index, messages
  bool sx = false;
  bool sx_valid = false;    // partial_d holds the owned nodes' totals and lf's bitmaps are exact
  bool gtot_valid = false;  // gtot = global totals of S_t (from the driver's all-reduce)
  bool sx_planned = false, sx_alld = false, sx_mid = false, last_sparse = false;
  uint32_t sx_maj = 0;
  std::vector<uint64_t> gtot;
  SxGeom sg{};
  SxBufs sb{};
  FrontierBufs lf{};
  void *lf_mem = nullptr, *sx_mem = nullptr;
  SxItem* rare_recv = nullptr;
  // sharded dense rounds on the binned pipeline (binned.h: SbGeom), else the direct kernels
  bool sbin = false;
  SbGeom sbg{};
  SbBufs sbb{};
  void* sb_mem = nullptr;
  bool sb_pre = false;  // gossip_dense_prepare ran for this round
  hipEvent_t ev_pre[2] = {};
  bool ev_pre_pending = false;
  SxItem* msg_recv = nullptr;
  uint64_t rare_recv_cap = 0, msg_recv_cap = 0, sx_stride = 0;
  // exchange dense rounds (binned.h: XdGeom), buffers allocated at the first one
  bool xd = false, xd_planned = false;
  uint32_t xd_shards = 6;  // gossip_set_param "xd_shards": G at which dense rounds become exchange rounds
  XdGeom xg{};
  XdBufs xb{};
  void *xd_smem = nullptr, *xd_rmem = nullptr;
  uint64_t xd_rcap = 0, xd_nin = 0;
  uint32_t* xd_cnt_h = nullptr;  // pinned [G]
  uint32_t xd_filt = 0;          // this round's edge filter (dense_filter of the global totals)
  bool xd_cls_ok = false;        // gossip_xd_classes handed out the own bitmaps for this round
  uint64_t* xd_cls = nullptr;    // [G][2 * nwl] every shard's occupancy bitmaps of S_t (all-gather in place)
  uint8_t* xd_keep = nullptr;    // [nown] per sender: the edges that survive the filter (count pass -> emit)
  // class-coded state exchange for dense image rounds (sharded.h cc_*), plan kind 4
  bool cc_planned = false;
  double cc_frac = 0.75;
  // replicated dense rounds (plan kinds 5 / 6): every rank runs the one-GPU binned
  // round over the whole state image in place, so the next dense round needs no collective
  // before it (kind 6) — where the links cost more than the extra device time (G = 2 at 2^27)
  int replicate = -1;           // gossip_set_param "replicate": -1 by the cost model, 0 never, 1 every dense round
  bool rep_planned = false;     // this round is replicated
  bool rep_img_ok = false;      // the image holds S_t of every node (the last round was replicated)
  BinGeom rbg{};
  BinBufs rbb{};
  void* rep_mem = nullptr;      // the one-GPU record slab over all N nodes, at the first replicated round
  uint64_t* rep_part = nullptr; // that round's whole-image totals (scratch: the ranks report own-slice totals)
  // gossip_set_param "link_gbps": sharded random-mode rounds pick sparse / dense by a per-rank
  // cost model with a link term (shard_round_costs); 0 = the fixed sparse_frac thresholds
  double link_gbps = 76.0;
  std::string model_plan;                // gossip_plan_model: this run's plan kinds, one letter per round
  double model_ms = 0, model_link_ms = 0;  // the modelled per-rank ms of the planned rounds since reset_timing
  uint64_t model_rounds = 0;
  double plan_cost[2] = {};  // the last plan's modelled sparse / dense ms (tools/shard_probe.py)  // gossip_set_param "cc_frac": at most this global fraction of mixed nodes
  uint64_t* cc_bits = nullptr;  // [G][cc_slot_words] every shard's bitmaps + prefix (all-gather in place)
  uint64_t* cc_vals = nullptr;  // [G][stride] the shards' mixed words
  uint64_t cc_vals_cap = 0, cc_stride = 0;
  uint64_t* sx_host = nullptr;  // pinned: [G + 2] counts / list bases
  uint64_t* pub_d = nullptr;    // device values for device-side collectives (gossip_*_dev): [G] counts, [1] count, partials

  hipEvent_t ev[kTimers][2] = {};
  double time_ms[kTimers] = {};
  uint64_t launches[kTimers] = {};
  bool timing = false;
  bool ev_pending[kTimers] = {};
  // per-round events of the pipelined rounds (timers 3 and 4), one pair per ring slot
  hipEvent_t evr[kRing][2] = {};
  int64_t evr_round[kRing] = {-1, -1, -1, -1, -1, -1, -1, -1};
  int evr_kind[kRing] = {};

  int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return code;
  }
};

#define HIP_OK(eng, expr)                                                                          \
  do {                                                                                             \
    hipError_t e_ = (expr);                                                                        \
    if (e_ != hipSuccess) return (eng)->fail(GOSSIP_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

namespace {

int set_dev(gossip_engine* e) {
  HIP_OK(e, hipSetDevice(e->device));
  if (e->ae_v_zero) {
    e->ae_v_zero = false;
    HIP_OK(e, hipMemsetAsync(e->V, 0, e->N * e->R * 4, e->stream));
  }
  return GOSSIP_OK;
}

// stats vector: [0] full [1] alive [2] messages [3] hash [4, 4+R) infected, [4+R] nonzero nodes (internal)
size_t part_len(const gossip_engine* e) { return 5 + (size_t)e->R; }

void free_all(gossip_engine* e) {
  uint64_t* bufs[] = {e->img[0], e->img[1], e->imgF, e->partial_d, e->scratch_d};
  if (e->mode == GOSSIP_MODE_FLOOD) {
    uint64_t* fb[] = {e->S, e->Snext, e->Sprev, e->skip};
    for (uint64_t* b : fb)
      if (b) (void)hipFree(b);
  }
  for (uint64_t* b : bufs)
    if (b) (void)hipFree(b);
  uint32_t* tb[] = {e->orow, e->ocol, e->irow, e->icol, e->fw.cur, e->fw.snd};
  for (uint32_t* b : tb)
    if (b) (void)hipFree(b);
  void* fe[] = {e->stall_d, e->fw.att};
  for (void* b : fe)
    if (b) (void)hipFree(b);
  if (e->bin_mem) (void)hipFree(e->bin_mem);
  if (e->rep_mem) (void)hipFree(e->rep_mem);
  if (e->rep_part) (void)hipFree(e->rep_part);
  if (e->fr_mem) (void)hipFree(e->fr_mem);
  void* sx[] = {e->lf_mem, e->sx_mem, e->rare_recv, e->msg_recv, e->sb_mem, e->xd_smem, e->xd_rmem,
                e->cc_bits, e->cc_vals, e->xd_cls, e->xd_keep};
  if (e->xd_cnt_h) (void)hipHostFree(e->xd_cnt_h);
  for (void* b : sx)
    if (b) (void)hipFree(b);
  if (e->sx_host) (void)hipHostFree(e->sx_host);
  if (e->pub_d) (void)hipFree(e->pub_d);
  if (e->ae_aux_alias) e->ae_aux = e->ae_aux_h = nullptr;  // inside partial_d / partial_h
  void* ae[] = {e->V, e->Vn, e->target, e->alive, e->alive_n, e->ae_aux, e->ae_claim, e->ae_eid, e->ae_erow, e->ae_segn, e->ae_pmask,
                e->ae_brec, e->ae_boff, e->ae_dboff, e->aex_img, e->aex_cnt, e->aex_boff, e->aex_bcnt, e->aex_req, e->aex_loc,
                e->aex_in, e->aex_resp_out, e->aex_resp_in, e->aex_tmp, e->aex_dirty, e->aex_verdict};
  if (e->aex_cnt_h) (void)hipHostFree(e->aex_cnt_h);
  for (void* b : ae)
    if (b) (void)hipFree(b);
  if (e->partial_h) (void)hipHostFree(e->partial_h);
  if (e->ae_aux_h) (void)hipHostFree(e->ae_aux_h);
  if (e->ae_slot_d) (void)hipFree(e->ae_slot_d);
  if (e->ae_gate_d) (void)hipFree(e->ae_gate_d);
  if (e->ae_slot_h) (void)hipHostFree(e->ae_slot_h);
  if (e->ring_h) (void)hipHostFree(e->ring_h);
  for (auto& p : e->ev)
    for (auto& x : p)
      if (x) (void)hipEventDestroy(x);
  for (auto& x : e->ev_pre)
    if (x) (void)hipEventDestroy(x);
  for (auto& x : e->wall_ev)
    if (x) (void)hipEventDestroy(x);
  for (auto& p : e->evr)
    for (auto& x : p)
      if (x) (void)hipEventDestroy(x);
  if (e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
}

RoundArgs make_args(gossip_engine* e, const uint64_t* gathered) {
  RoundArgs a{};
  a.S = e->S;
  a.G = gathered;
  a.Snext = e->Snext;
  a.partial = e->partial_d;
  a.N = e->N;
  a.Nl = e->Nl;
  a.lo = e->lo;
  a.nown = e->nown;
  a.W = e->W;
  a.R = e->R;
  a.k = e->k;
  a.t = e->t;
  a.key0 = e->key0;
  a.key1 = e->key1;
  a.fa = e->fa;
  a.flags = e->cfg.flags;
  a.mode = e->mode;
  a.Sprev = e->Sprev;
  a.skip = e->skip;
  a.orow = e->orow;
  a.ocol = e->ocol;
  a.irow = e->irow;
  a.icol = e->icol;
  return a;
}

int timer_begin(gossip_engine* e, int which) {
  if (!e->timing) return GOSSIP_OK;
  HIP_OK(e, hipEventRecord(e->ev[which][0], e->stream));
  return GOSSIP_OK;
}

int timer_end(gossip_engine* e, int which) {
  if (!e->timing) return GOSSIP_OK;
  HIP_OK(e, hipEventRecord(e->ev[which][1], e->stream));
  e->ev_pending[which] = true;
  return GOSSIP_OK;
}

// called after a stream sync: fold finished event pairs into the totals
// count = false: a piece of a round whose last piece counts the launch (exchange rounds
// time their three engine calls, not the collectives between them)
int timer_collect(gossip_engine* e, bool count = true) {
  if (!e->timing) return GOSSIP_OK;
  for (int w = 0; w < kTimers; ++w) {
    if (!e->ev_pending[w]) continue;
    float ms = 0.f;
    HIP_OK(e, hipEventElapsedTime(&ms, e->ev[w][0], e->ev[w][1]));
    e->time_ms[w] += ms;
    e->launches[w] += count ? 1 : 0;
    e->ev_pending[w] = false;
  }
  if (e->ev_pre_pending) {  // the prepared part of a dense sharded round counts with timer 0
    float ms = 0.f;
    HIP_OK(e, hipEventElapsedTime(&ms, e->ev_pre[0], e->ev_pre[1]));
    e->time_ms[0] += ms;
    e->ev_pre_pending = false;
  }
  return GOSSIP_OK;
}

AexArgs make_aex_args(gossip_engine* e);

// exchange payload for this round: S_t (random modes) or F_t (FLOOD); the
// send slice lies inside the gathered image, so the all-gather is in place.
int prepare_send(gossip_engine* e, uint64_t** send, uint64_t** image) {
  if (e->aex) {  // sharded ANTIENTROPY: the own {alive, stale} word pairs into every shard's image
    if (e->aex_churned != e->t) {  // the own nodes' churn of round t, once
      HIP_OK(e, launch_aex_churn(make_aex_args(e), e->stream));
      e->aex_churned = e->t;
    }
    *send = e->aex_img + (size_t)e->rank * e->Nl / 32;
    *image = e->aex_img;
    return GOSSIP_OK;
  }
  if (e->mode == GOSSIP_MODE_ANTIENTROPY) {  // single shard: nothing to exchange
    *send = *image = nullptr;
    return GOSSIP_OK;
  }
  if (e->mode == GOSSIP_MODE_FLOOD) {
    HIP_OK(e, launch_frontier(e->S, e->Sprev, e->F, (uint64_t)e->W * e->Nl, e->stream));
    *send = e->F;
    *image = e->imgF;
  } else {
    *send = e->S;
    *image = e->img[e->cur];
  }
  return GOSSIP_OK;
}

uint64_t* current_image(gossip_engine* e) { return e->mode == GOSSIP_MODE_FLOOD ? e->imgF : e->img[e->cur]; }

void bind_slices(gossip_engine* e) {
  const size_t off = (size_t)e->rank * e->W * e->Nl;
  if (e->mode == GOSSIP_MODE_ANTIENTROPY) return;
  if (e->mode == GOSSIP_MODE_FLOOD) {
    e->F = e->imgF + off;
  } else {
    e->S = e->img[e->cur] + off;
    e->Snext = e->img[e->cur ^ 1] + off;
  }
}

AeArgs make_ae_args(gossip_engine* e) {
  AeArgs a{};
  a.V = e->V;
  a.Vn = e->Vn;
  a.ab = e->alive;
  a.abn = e->alive_n;
  a.target = e->target;
  a.partial = e->partial_d;
  a.N = e->N;
  a.K = e->R;
  a.L = ae_lanes(e->R);
  a.k = e->k;
  a.t = e->t;
  a.key0 = e->key0;
  a.key1 = e->key1;
  a.fail = e->cfg.churn_fail;
  a.rec = e->cfg.churn_recover;
  a.flags = e->cfg.flags;
  a.aux = e->ae_aux;
  a.eid = e->ae_eid;
  a.erow = e->ae_erow;
  a.claim = e->ae_claim;
  a.segn = e->ae_segn;
  a.pmask = e->ae_pmask;
  a.nseg = e->ae_nseg;
  a.spc = e->ae_spc;
  a.segcap = e->ae_segcap;
  a.brec = e->ae_brec;
  a.boff = e->ae_boff;
  a.btl = e->ae_bg.tl;
  a.bnt = e->ae_bg.nt;
  a.brs = e->ae_bg.rs;
  a.bnreg = e->ae_bg.nreg;
  a.spb = std::max<uint32_t>(1, 4096 / e->ae_nseg);  // ~4096 blocks over the edge list
  a.epoch = e->ae_epoch;
  return a;
}

// Device time (ms) per launch of `run` on the engine's stream: the average of two after a warm-up.
template <class Run>
int timed_trial(gossip_engine* e, Run run, float* ms) {
  hipEvent_t ev[2];
  HIP_OK(e, hipEventCreate(&ev[0]));
  HIP_OK(e, hipEventCreate(&ev[1]));
  bool ok = true;
  for (int i = 0; i < 3 && ok; ++i) {
    if (i == 1) ok = hipEventRecord(ev[0], e->stream) == hipSuccess;
    if (ok) ok = run() == hipSuccess;
  }
  ok = ok && hipEventRecord(ev[1], e->stream) == hipSuccess && hipEventSynchronize(ev[1]) == hipSuccess &&
       hipEventElapsedTime(ms, ev[0], ev[1]) == hipSuccess;
  *ms *= 0.5f;
  (void)hipEventDestroy(ev[0]);
  (void)hipEventDestroy(ev[1]);
  return ok ? GOSSIP_OK : e->fail(GOSSIP_EHIP, "placement trial round failed");
}

// Placement of a slab: `trial(slab, &ms)` times a round over the slab at `slab`;
// up to place_tries allocations of `bytes` are tried and the fastest is kept in *mem.  At most two
// slabs are held beside the kept one: the best so far, the last loser (held while the next
// candidate is allocated, so that candidate cannot reuse its pages) and the new candidate
// (round 5 held every candidate: 75 GB at 2^27).  Timer 5 gets the trial rounds.  Returns whether
// *mem moved.
template <class Trial>
int place_slab(gossip_engine* e, void** mem, size_t bytes, Trial trial, bool* moved, const char* what) {
  *moved = false;
  // A wall-time budget: on some boxes and processes a fresh multi-GiB hipMalloc / hipFree takes
  // 0.1 s to seconds instead of milliseconds (a 3.3 s first step at 2^27 where 130 ms is usual,
  // with the trials' device time unchanged at 66 ms): past it no further candidate
  // is tried and the best so far is kept.  (400 ms cut such a box's lottery to 2-5 candidates and
  // left 2 of 4 engines in the 5.5-ms mode, profiles/r06_vmm/budget400)
  constexpr double kPlaceBudgetMs = 2000.0;
  const auto t_start = std::chrono::steady_clock::now();
  void* best = *mem;
  void* held = nullptr;
  float best_ms = 0.f;
  int rc = trial(best, &best_ms);
  auto account = [&](float ms) {
    e->time_ms[5] += 3.0 * ms;
    e->launches[5] += 3;
  };
  account(best_ms);
#ifdef GOSSIP_EXP_PLACE_LOG
  std::fprintf(stderr, "%s: candidate 0 slab %p trial %.1f us\n", what, best, best_ms * 1e3);
#endif
  for (uint32_t i = 1; i < e->place_tries && rc == GOSSIP_OK; ++i) {
    if (std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count() > kPlaceBudgetMs)
      break;
    void* p = nullptr;
#ifdef GOSSIP_EXP_PLACE_LOG
    const auto t0 = std::chrono::steady_clock::now();
#endif
    if (hipMalloc(&p, bytes) != hipSuccess) {
      (void)hipGetLastError();  // no room for another trial: keep the best so far
      break;
    }
#ifdef GOSSIP_EXP_PLACE_LOG
    const auto t1 = std::chrono::steady_clock::now();
#endif
    float ms = 0.f;
    rc = trial(p, &ms);
    account(ms);
#ifdef GOSSIP_EXP_PLACE_LOG
    std::fprintf(stderr, "%s: candidate %u slab %p trial %.1f us, hipMalloc %.1f ms\n", what, i, p, ms * 1e3,
                 std::chrono::duration<double, std::milli>(t1 - t0).count());
#endif
    void* loser = p;
    if (rc == GOSSIP_OK && ms < best_ms) {
      loser = best;
      best = p;
      best_ms = ms;
    }
#ifdef GOSSIP_EXP_PLACE_LOG
    const auto t2 = std::chrono::steady_clock::now();
#endif
    if (held) (void)hipFree(held);  // (its trial has completed: timed_trial synchronizes)
#ifdef GOSSIP_EXP_PLACE_LOG
    std::fprintf(stderr, "%s: hipFree %.1f ms\n", what,
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t2).count());
#endif
    held = loser;
  }
  (void)what;
  if (held) (void)hipFree(held);
  *moved = best != *mem;
  *mem = best;
  return rc;
}

// One placement candidate's trial (place_bins, rep_compute): one emit over the image `img` (read
// only) fills the candidate's records, then serve alone is timed, its tile queues cleared before
// each launch.  The slab's mode is serve's (the trial round follows bin_serve at r = 0.93-0.99
// across candidates); whole trial rounds chose equally fast slabs at twice the
// cost (first step at 2^27 230 vs 127 ms, profiles/r06_vmm/place_serve).
int serve_trial(gossip_engine* e, const BinGeom& g, bool dyn, void* slab, uint64_t* img, uint64_t* part, float* ms) {
  BinBufs b{};
  bin_carve(g, slab, &b);
  b.nzb = b.fullb = nullptr;
  if (!dyn) b.dyn = nullptr;
  if (b.dyn) HIP_OK(e, hipMemsetAsync(b.dyn, 0, 17 * 4, e->stream));
  const RoundSync rs{nullptr, (uint32_t)part_len(e), 0u};
  auto part_round = [&](uint32_t parts) {
    return launch_binned_round(g, b, img, part, e->R, 0u, e->key0, e->key1, e->mode, 0u, Faults{}, 0u, rs,
                               e->stream, parts);
  };
  HIP_OK(e, part_round(1u));
  return timed_trial(e, [&] {
    if (b.dyn) {
      if (hipError_t x = hipMemsetAsync(b.dyn, 0, 16 * 4, e->stream)) return x;
    }
    return part_round(2u);
  }, ms);
}

// Before the first round of a binned engine with a record slab of 512 MiB or more: its placement
// (place_slab), each trial a dense round on a zero state (the second image, unused by the in-place
// binned rounds) with scratch totals and no bitmaps.
int place_bins(gossip_engine* e) {
  if (e->placed) return GOSSIP_OK;
  e->placed = true;
  const size_t bytes = bin_bytes(e->bg);
  auto recarve = [&]() -> int {
    BinBufs nb{};
    bin_carve(e->bg, e->bin_mem, &nb);
    nb.nzb = e->bb.nzb;
    nb.fullb = e->bb.fullb;
    HIP_OK(e, hipMemset(nb.dyn, 0, 17 * 4));
    e->bb_dyn = nb.dyn;
    if (!e->bb.dyn) nb.dyn = nullptr;
    e->bb = nb;
    return GOSSIP_OK;
  };
  if (!e->binned || e->place_tries <= 1 || bytes < (512ull << 20) || !e->img[1]) return GOSSIP_OK;
  uint64_t* part = nullptr;
  HIP_OK(e, hipMalloc((void**)&part, (part_len(e) + 8) * 8));
  bool moved = false;
  const int rc = place_slab(e, &e->bin_mem, bytes, [&](void* slab, float* ms) {
    return serve_trial(e, e->bg, e->bb.dyn != nullptr, slab, e->img[1], part, ms);
  }, &moved, "place_bins");
  (void)hipFree(part);
  if (moved) {
    const int r2 = recarve();
    return rc != GOSSIP_OK ? rc : r2;
  }
  return rc;
}

// A sharded engine's dense-round slab (the state all-gather rounds' push and pull passes, sb_*)
// the same way, before its first such round: each trial a round over the current image into a
// scratch slice with scratch totals and no bitmaps (image read only).
int place_sb(gossip_engine* e) {
  if (e->sb_placed) return GOSSIP_OK;
  e->sb_placed = true;
  const size_t bytes = sb_bytes(e->sbg);
  if (!e->sbin || e->place_tries <= 1 || bytes < (512ull << 20)) return GOSSIP_OK;
  uint64_t *part = nullptr, *snext = nullptr;
  HIP_OK(e, hipMalloc((void**)&part, (part_len(e) + 8) * 8));
  if (hipMalloc((void**)&snext, std::max<uint64_t>(e->nown, 1) * 8) != hipSuccess) {
    (void)hipFree(part);
    return e->fail(GOSSIP_ENOMEM, "placement scratch allocation failed");
  }
  bool moved = false;
  const uint64_t* image = current_image(e);
  const int rc = place_slab(e, &e->sb_mem, bytes, [&](void* slab, float* ms) {
    SbBufs b{};
    sb_carve(e->sbg, slab, &b);
    return timed_trial(e, [&] {
      if (hipError_t x = hipMemsetAsync(part, 0, part_len(e) * 8, e->stream)) return x;
      return launch_sb_round(e->sbg, b, image, snext, part, e->R, e->t, e->key0, e->key1, e->mode, Faults{}, 0u,
                             nullptr, nullptr, e->stream);
    }, ms);
  }, &moved, "place_sb");
  (void)hipStreamSynchronize(e->stream);
  (void)hipFree(part);
  (void)hipFree(snext);
  if (moved) sb_carve(e->sbg, e->sb_mem, &e->sbb);
  return rc;
}

// Binned engines: make partial_d hold the exact totals of S (and the bitmaps
// exact) when an untracked write (plain inject) left them stale.
int prepare_planned(gossip_engine* e) {
  if (int rc = place_bins(e)) return rc;
  if (!e->frontier || e->fr_valid) return GOSSIP_OK;
  HIP_OK(e, hipMemsetAsync(e->partial_d, 0, part_len(e) * 8, e->stream));
  HIP_OK(e, launch_frontier_rebuild(e->fb, e->S, e->N, e->partial_d, e->R, e->cfg.flags, e->stream));
  e->fr_valid = true;
  return GOSSIP_OK;
}

// Totals the path choice needs: full and nonzero counts, per-rumor infected.
struct Est {
  double full = 0, nz = 0;
  std::vector<double> inf;
};

Est est_of(const gossip_engine* e, const uint64_t* tot) {
  Est x;
  x.full = (double)tot[0];
  x.nz = (double)tot[4 + e->R];
  x.inf.assign(tot + 4, tot + 4 + e->R);
  return x;
}

// One round of the mean-field model of the random modes, per rumor: a node
// misses rumor r after the round iff it held no copy, none of its k pulls hit a
// holder (u^k) and no holder pushed to it (e^{-k(1-u)}).  Only steers the path
// choice, never a result.
Est predict(const gossip_engine* e, const Est& x) {
  Est y;
  // lost edges (§2.8) thin the fanout; a partition keeps ~1/P of the peers
  const double keep = (1.0 - (double)e->fa.loss / 4294967296.0) * (e->fa.parts > 1 ? 1.0 / e->fa.parts : 1.0);
  const double N = (double)e->N, k = (double)e->k * keep;
  const bool push = e->mode == GOSSIP_MODE_PUSH || e->mode == GOSSIP_MODE_PUSHPULL;
  const bool pull = e->mode == GOSSIP_MODE_PULL || e->mode == GOSSIP_MODE_PUSHPULL;
  double all_miss = 1.0, all_hit = 1.0;
  y.inf.resize(x.inf.size());
  for (size_t r = 0; r < x.inf.size(); ++r) {
    const double u = 1.0 - x.inf[r] / N;
    double v = u;
    if (pull) v *= std::pow(u, k);
    if (push) v *= std::exp(-k * (1.0 - u));
    y.inf[r] = (1.0 - v) * N;
    all_miss *= v;
    all_hit *= 1.0 - v;
  }
  y.nz = N * (1.0 - all_miss);
  y.full = N * all_hit;
  return y;
}

// the sparse-round threshold: gossip_set_param's, else the default of the engine's dense
// round kind — a sharded dense round that all-gathers the state costs more than an
// exchange round, so sparse rounds pay off up to a larger rare fraction before it
// (tools/shard_probe.py sweeps, profiles/r02_xd)
double sparse_frac_of(const gossip_engine* e) {
  if (e->sparse_frac_set || !e->sx) return e->sparse_frac;
  // before exchange rounds: 1/25 (a round with ~5 % rare nodes is cheaper as a class-filtered
  // exchange round, profiles/r02_xdfilt/); before state all-gathers: 1/4
  return e->xd && e->xd_shards && e->G >= e->xd_shards ? 0.04 : 0.25;
}

// Per-rank cost model of one sharded round of the random modes, in ms: device time from the
// measured rates plus link time = the bytes the rank sends over its links /
// (link_gbps x the G - 1 links it uses, at most 7).  Only steers the plan (every kind computes
// the same bits).  Device rates: a sparse round costs 2.3 ps per own node (the Philox floor; round
// 0 at 2^27 on one GPU: 311 us) plus up to 70 ps per own node as the rare share r grows, x (1 -
// e^(-r / 0.05)) (the summaries saturate: G = 2 x 2^26 at r = 3.7 / 19 / 25 %: 2.41 / 5.0 / 4.83 ms,
// profiles/r05_shard/probe_G2_fixed.txt); a dense round on the state image 7.3 ps per image node + 47 ps per own node (N = 2 / 4
// ranks x 2^26 / 2^25: 4.14 / 2.56 ms, profiles/r04_ad/); an exchange round 67 ps per own node
// (G = 8 x 2^24: 1.13 ms, profiles/r02_xd/).  Link bytes per rank: sparse = the rare-list
// all-gather (16 B per rare node of the shard to each other shard) + the off-shard pushes
// (16 B items, ~k per rare node); state all-gather = 8 B per own node to each other shard
// (class-coded: its bitmaps + prefixes, 20 B per 64 nodes, + 8 B per mixed node); exchange =
// 40 (G - 1) / G B per own node (12-B items out, 8-B replies back, k = 2).
struct ShardCosts {
  double sparse, dense;            // modelled ms per rank: device + link
  double sparse_link, dense_link;  // their link parts
  bool dense_xd, dense_cc;
  // a replicated dense round (kinds 5 / 6): device time of the one-GPU round over
  // all N nodes (5.1 ms at 2^27 on MI355X: 3.8e-8 ms per node) plus the own-slice totals, and the
  // state all-gather when the image is not whole yet (kind 5)
  double rep, rep_link;
  bool rep_ok;
};
uint32_t dense_filter(const gossip_engine* e, const Est& x, double frac);

ShardCosts shard_round_costs(const gossip_engine* e, const Est& x) {
  // (Nl, not the own count: every rank must reach the same plan, also with ragged shards)
  const double N = (double)e->N, G = (double)e->G, Nl = (double)e->Nl, k = (double)e->k;
  const double rare = std::min(x.nz, N - x.full), rare_own = rare / G;
  const double bw = e->link_gbps * 1e6 * std::min(G - 1.0, 7.0);  // bytes per ms
  ShardCosts c{};
  c.sparse_link = (16.0 * rare_own * (G - 1.0) + 16.0 * k * rare_own * (G - 1.0) / G) / bw;
  c.sparse = Nl * (2.3e-9 + 7.0e-8 * (1.0 - std::exp(-rare / N / 0.05))) + c.sparse_link;
  c.dense_xd = e->xd && e->xd_shards && e->G >= e->xd_shards;
  const double mixed = std::max(0.0, x.nz - x.full);
  c.dense_cc = !c.dense_xd && e->cc_frac > 0 && mixed / N <= e->cc_frac;
  if (c.dense_xd) {
    // items per own sender edge that survive the class filter (gossip_xd_classes, dense_filter of
    // these totals): a pull-only edge (empty sender) into an empty peer and a push-only one (full
    // sender) into a full peer are never sent.  Device time fitted on the G = 8 probe (unfiltered
    // 1.15 ms, filtered at 34 % kept 0.93 ms per 2^24-node rank, profiles/r05_probes/); round 4's
    // model priced every round unfiltered and planned the two filtered rounds sparse (1.6-1.7 ms)
    const uint32_t filt = e->k <= 8 ? dense_filter(e, x, e->xd_filter_frac) : 0u;
    const double ef = 1.0 - x.nz / N, ff = x.full / N, mf = std::max(0.0, 1.0 - ef - ff);
    const double kept = mf + ef * ((filt & 1u) ? 1.0 - ef : 1.0) + ff * ((filt & 2u) ? 1.0 - ff : 1.0);
    c.dense_link = 40.0 * (G - 1.0) / G * Nl * kept / bw;
    c.dense = Nl * (4.85e-8 + 2.0e-8 * kept) + c.dense_link;
  } else {
    const double slice = c.dense_cc ? 20.0 / 64.0 * Nl + 8.0 * mixed / G : 8.0 * Nl;
    c.dense_link = slice * (G - 1.0) / bw;
    c.dense = 7.3e-9 * N + 4.7e-8 * Nl + c.dense_link;
  }
  c.rep_ok = e->replicate != 0 && e->sx && bin_path_ok(e->N, e->k, 1, 1);
  // entering gathers the image class-coded where the dense round would (kind 7), else whole (5)
  const double cc_slice = 20.0 / 64.0 * Nl + 8.0 * mixed / G;
  c.rep_link = e->rep_img_ok ? 0.0 : (c.dense_cc ? cc_slice : 8.0 * Nl) * (G - 1.0) / bw;
  c.rep = 3.8e-8 * N + 1.5e-9 * Nl + c.rep_link;
  return c;
}

// What replicating saves over the dense rounds after this one (kind 6 instead of a sharded dense
// round each), as far as the mean-field predictor sees them: up to 8 rounds, until one that the
// model would run sparse.  Only steers the plan.
double rep_gain_ahead(const gossip_engine* e, Est x) {
  double gain = 0.0;
  for (int i = 0; i < 8; ++i) {
    x = predict(e, x);
    const ShardCosts c = shard_round_costs(e, x);
    const double rep6 = c.rep - c.rep_link;
    if (c.sparse < std::min(c.dense, rep6)) break;  // the dense phase ends
    gain += std::max(0.0, c.dense - rep6);
  }
  return gain;
}

// sparse when the smaller rare class is at most sparse_frac * N; maj = which
// class is rare; all_d once the rare ends' pushes (~k per rare node) reach
// alld_frac * N (launch_frontier_round)
bool choose_sparse(const gossip_engine* e, const Est& x, uint32_t* maj, bool* all_d) {
  if (!e->frontier && !e->sx) return false;
  const double lo = x.nz, hi = (double)e->N - x.full, rare = std::min(lo, hi);
  *maj = hi < lo ? 1u : 0u;
  *all_d = rare * (double)e->k >= e->alld_frac * (double)e->N;
  return rare <= sparse_frac_of(e) * (double)e->N;
}

// the binned sparse scan: once the LDS summary (g nodes per bit) would have a bit set under
// 1 - (1 - r)^g >= bscan_frac of the peers it filters too little, and binning every edge by peer
// tile costs less than probing the mid-level summary and the exact bitmap per edge (DESIGN.md
// §3.3).  Its records and run table live in the dense round's record slab.
bool bscan_round(const gossip_engine* e, const Est& x, uint32_t maj) {
  if (!e->binned || !e->frontier || !bs_path_ok(e->N, e->k) || e->bscan_frac > 1.0) return false;
  const size_t recs = (size_t)e->bg.nt_s * e->bg.rp;
  if (bs_rec_bytes(e->N, e->k) > recs * 8 || bs_tab_bytes(e->N) > recs * 8) return false;
  if (e->bscan_frac <= 0.0) return true;
  // by default only where the LDS summary is coarse (g >= 64 nodes per bit: past 2^25 nodes, where
  // the mid-level summary exists); at 2^24 the one heavy sparse round it took ran 590 us and the
  // step's sparse rounds 1.10 -> 1.44 ms (K1b has too few regions per tile to fill its waves)
  if (!e->fb.summ2) return false;
  const double N = (double)e->N, rare = maj ? N - x.full : x.nz;
  const double g = (double)(1u << e->fb.glog);
  return 1.0 - std::pow(1.0 - std::min(std::max(rare / N, 0.0), 1.0), g) >= e->bscan_frac;
}

// dense rounds: probe the peer's class in emit when many edges would move
// nothing (pulls from empty peers early in a run, pushes into full peers late)
uint32_t dense_filter(const gossip_engine* e, const Est& x, double frac) {
  const double N = (double)e->N, empty = 1.0 - x.nz / N, full = x.full / N;
  const bool pull = e->mode == GOSSIP_MODE_PULL || e->mode == GOSSIP_MODE_PUSHPULL;
  const bool push = e->mode == GOSSIP_MODE_PUSH || e->mode == GOSSIP_MODE_PUSHPULL;
  return (pull && empty > frac ? 1u : 0u) | (push && full > frac ? 2u : 0u);
}

// the one-shard dense filter's threshold: gossip_set_param's, else 0.3 while the occupancy
// bitmaps (N/8 bytes each) fit an XCD's 4 MiB L2; past that every probe is a 64-B fetch from
// the MALL or HBM and the probes cost more than the edges they drop (2^27 nodes: emit
// 2.3 -> 6.3 ms, serve + apply -1.6 ms; profiles/r03_a/rounds.txt)
double filter_frac_of(const gossip_engine* e) {
  if (e->filter_frac_set) return e->filter_frac;
  return e->N <= (1ull << 25) ? e->filter_frac : 2.0;
}

RoundSync ring_sync(gossip_engine* e, uint32_t slot) {
  RoundSync rs;
  rs.ring = e->ring_d + (size_t)slot * (part_len(e) + 1);
  rs.plen = (uint32_t)part_len(e);
  rs.seq = (uint32_t)++e->seq;
  return rs;
}

// Folds the per-round events of ring slot `slot` into timer 3 (dense) or 4
// (sparse) when that round is below `limit` (rounds enqueued past convergence
// are not counted).
int round_timer_collect(gossip_engine* e, uint32_t slot, int64_t limit) {
  if (e->evr_round[slot] < 0) return GOSSIP_OK;
  HIP_OK(e, hipEventSynchronize(e->evr[slot][1]));
  if (e->evr_round[slot] < limit) {
    float ms = 0.f;
    HIP_OK(e, hipEventElapsedTime(&ms, e->evr[slot][0], e->evr[slot][1]));
    e->time_ms[e->evr_kind[slot]] += ms;
    e->launches[e->evr_kind[slot]] += 1;
  }
  e->evr_round[slot] = -1;
  return GOSSIP_OK;
}

// One pipelined round: its kernels (bracketed by the slot's events when timing),
// then the snapshot of the totals into ring slot `slot` (rs).
int launch_round_path(gossip_engine* e, uint32_t t, bool sparse, uint32_t maj, bool all_d, uint32_t filt,
                      const RoundSync& rs, int slot, bool bscan) {
  const bool timed = e->timing && slot >= 0;
  if (timed) {
    if (int rc = round_timer_collect(e, (uint32_t)slot, INT64_MAX)) return rc;
    HIP_OK(e, hipEventRecord(e->evr[slot][0], e->stream));
  }
  // the mid-level summary (FrontierBufs::summ2) pays once many peers hit the LDS summary (a
  // g-node group holds a rare node w.p. 1 - (1 - r)^g); below that its extra probe round trip
  // costs more than the exact probes it saves (2^27 nodes: rounds at 1-17 % LDS hits +50..130 us,
  // at 61 % -920 us; profiles/r03_mid).  The kernels decide from the exact rare count.
  FrontierBufs fb = e->fb;
  fb.mid_frac = (float)e->mid_frac;
  if (sparse && bscan) {  // (the slab pointers change when placement re-carves it)
    fb.brec = (uint32_t*)e->bb.resp;
    fb.btab = (uint16_t*)(e->bb.prec ? (void*)e->bb.prec : (void*)e->bb.vals);
    fb.btiles = bs_tiles(e->N);
    fb.bregions = bs_regions(e->N);
    fb.btabT = fb.btab + bs_tab_bytes(e->N) / 4;  // (the second half of bs_tab_bytes)
  }
  if (sparse)
    HIP_OK(e, launch_frontier_round(fb, e->S, e->N, e->partial_d, e->R, e->k, t, e->key0, e->key1, e->mode, maj,
                                    !all_d ? kSparseFlags : (maj == 0 && e->sparse_direct ? kSparseDirect : kSparseAllD),
                                    e->fa, e->cfg.flags, rs, e->stream));
  else
    HIP_OK(e, launch_binned_round(e->bg, e->bb, e->S, e->partial_d, e->R, t, e->key0, e->key1, e->mode, filt,
                                  e->fa, e->cfg.flags, rs, e->stream));
  if (timed) {
    HIP_OK(e, hipEventRecord(e->evr[slot][1], e->stream));
    e->evr_round[slot] = t;
    e->evr_kind[slot] = sparse ? 4 : 3;
  }
  HIP_OK(e, launch_round_snapshot(e->partial_d, rs, e->stream));
  // stall streaks after round t (gossip_round_commit does it for rounds not run from here)
  if (e->stall_d && slot >= 0)
    HIP_OK(e, launch_stall_update(e->stall_d, e->N, e->k, t, e->key0, e->key1, e->fa, e->stream));
  return GOSSIP_OK;
}

// Waits until ring slot `slot` carries sequence `want` (the round's last block
// wrote it), polling host memory; a stream error ends the wait.
int wait_slot(gossip_engine* e, uint32_t slot, uint64_t want) {
  volatile uint64_t* sq = e->ring_h + (size_t)slot * (part_len(e) + 1) + part_len(e);
  for (uint64_t spin = 0; *sq != want; ++spin) {
    _mm_pause();
    if ((spin & 4095) == 4095) {
      const hipError_t q = hipStreamQuery(e->stream);
      if (q != hipSuccess && q != hipErrorNotReady)
        return e->fail(GOSSIP_EHIP, "round kernels failed: %s", hipGetErrorString(q));
      if (q == hipSuccess && *sq != want) return e->fail(GOSSIP_EHIP, "round %llu never reported",
                                                        (unsigned long long)want);
    }
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return GOSSIP_OK;
}

int read_totals(gossip_engine* e, std::vector<uint64_t>* out) {
  HIP_OK(e, hipMemcpyAsync(e->partial_h, e->partial_d, part_len(e) * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  out->assign(e->partial_h, e->partial_h + part_len(e));
  return GOSSIP_OK;
}

// gossip_step for binned engines.  Round r's path is chosen from the last totals
// read (S after round done-1) predicted forward over the rounds still in
// flight; rounds past convergence find nothing rare and return at once, and are
// not counted.  Timer 0 brackets the whole step (per-round device time
// including the gaps between rounds).
int step_planned(gossip_engine* e, uint32_t max_rounds, gossip_round_stats_t* stats, uint64_t* infected,
                 uint32_t* rounds_done) {
  if (int rc = prepare_planned(e)) return rc;
  std::vector<uint64_t> t0tot;
  if (int rc = read_totals(e, &t0tot)) return rc;
  Est base = est_of(e, t0tot.data());
  const size_t pl = part_len(e);
  const uint32_t t0 = e->t;
  std::vector<uint64_t> want(kRing, 0);
  uint32_t launched = 0, done = 0;
  bool stop = false;
  // the stall streaks are not idempotent: a round enqueued past convergence would
  // advance them for a round the next step runs again, so stall engines run one
  // round ahead only
  const uint32_t ahead = e->stall_d ? 1u : e->ahead;
  if (e->timing) HIP_OK(e, hipEventRecord(e->ev[0][0], e->stream));
  while (done < max_rounds) {
    while (!stop && launched < max_rounds && launched - done < ahead) {
      Est x = base;
      for (uint32_t i = done; i < launched; ++i) x = predict(e, x);
      uint32_t maj = 0;
      bool all_d = false;
      const bool sparse = choose_sparse(e, x, &maj, &all_d);
      const uint32_t filt = dense_filter(e, x, filter_frac_of(e));
      const uint32_t slot = launched % kRing;
      const RoundSync rs = ring_sync(e, slot);
      want[slot] = rs.seq;
      if (int rc = launch_round_path(e, t0 + launched, sparse, maj, all_d, filt, rs, (int)slot,
                                     sparse && bscan_round(e, x, maj)))
        return rc;
      ++launched;
    }
    if (done == launched) break;
    const uint32_t slot = done % kRing;
    if (int rc = wait_slot(e, slot, want[slot])) return rc;
    const uint64_t* tot = e->ring_h + (size_t)slot * (pl + 1);
    gossip_round_stats_t st;
    st.round = t0 + done;
    st.full_nodes = tot[0];
    st.alive_nodes = e->N;
    st.converged = tot[0] == e->N ? 1u : 0u;
    st.messages = 0;
    st.state_hash = (e->cfg.flags & GOSSIP_FLAG_HASH) ? tot[3] : 0;
    if (stats) stats[done] = st;
    if (infected) std::memcpy(infected + (size_t)done * e->R, tot + 4, (size_t)e->R * 8);
    base = est_of(e, tot);
    ++done;
    if (st.converged) stop = true;
    if (stop) break;
  }
  if (e->timing) HIP_OK(e, hipEventRecord(e->ev[0][1], e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  if (e->timing) {
    float ms = 0.f;
    HIP_OK(e, hipEventElapsedTime(&ms, e->ev[0][0], e->ev[0][1]));
    e->time_ms[0] += ms;
    e->launches[0] += done;
    for (uint32_t s = 0; s < kRing; ++s)
      if (int rc = round_timer_collect(e, s, (int64_t)t0 + done)) return rc;
  }
  e->t = t0 + done;
  if (rounds_done) *rounds_done = done;
  return GOSSIP_OK;
}

// ANTIENTROPY round.  Sparse (in place) when the stale
// bitmap is valid and the exchanges touching a stale node are predicted to fit
// the edge list; a list that overflowed leaves V, the bitmap and the claims
// untouched, and the round is rerun dense.  Stats reach the host every round.
int ae_read_back(gossip_engine* e) {
  HIP_OK(e, hipMemcpyAsync(e->partial_h, e->partial_d, (part_len(e) + 2) * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  return GOSSIP_OK;
}

bool ae_plan_sparse(const gossip_engine* e) {
  if (!e->ae_sb_valid || e->ae_force == 0 || e->ae_dense_next) return false;
  if (e->ae_force == 1) return true;
  // exchanges with a stale end ~ 2k x (alive stale after churn): the alive stale
  // nodes that survive plus the stale dead ones that revive (x1.5 margin)
  const double alive_stale = (double)(e->ae_alive - e->ae_full);
  const double dead_stale = std::max(0.0, (double)e->ae_stale - alive_stale);
  const double rec = e->cfg.churn_recover / 4294967296.0;
  const double pred = 3.0 * e->k * (alive_stale + dead_stale * rec) + 1024.0;
  return pred <= 0.7 * (double)e->ae_cap;  // the largest segment, not the mean, must fit
}

// One-engine ANTIENTROPY, before its first dense round: the same placement choice as place_bins
// for the rows (V, Vn), which the dense apply gathers from, over place_tries candidates.
// Each candidate gets a copy of the rows; its trial is a dense round of the current state into its
// own Vn with scratch totals (the real round rewrites everything the trial wrote).
int ae_place(gossip_engine* e) {
  e->ae_placed = true;
  const size_t vb = (size_t)e->N * e->R * 4;
  if (e->place_tries <= 1 || !(e->ae_dbin && e->ae_dbin_on) || vb < (512ull << 20)) return GOSSIP_OK;
  const size_t pl = part_len(e);
  uint64_t* part = nullptr;
  HIP_OK(e, hipMalloc((void**)&part, (pl + 8) * 8));
  struct Cand {
    uint32_t *V, *Vn;
  };
  // (as place_slab: the kept rows, the best candidate so far, the last loser held while the next
  // candidate is allocated, and that candidate: at most two sets of rows beside the kept ones)
  Cand best{e->V, e->Vn}, held{nullptr, nullptr};
  float best_ms = 0.f;
  hipEvent_t ev[2];
  HIP_OK(e, hipEventCreate(&ev[0]));
  HIP_OK(e, hipEventCreate(&ev[1]));
  int rc = GOSSIP_OK;
  auto release = [](Cand& c) {
    if (c.V) (void)hipFree(c.V);
    if (c.Vn) (void)hipFree(c.Vn);
    c = Cand{nullptr, nullptr};
  };
  const uint32_t tries = e->place_tries;  // 12 by default: a fast placement of the rows is ~1 in 8
  for (uint32_t i = 0; i < tries && rc == GOSSIP_OK; ++i) {
    Cand c = best;
    if (i > 0) {
      // the rows carry the mode, the records do not (profiles/r05_pl/r05_aem/): only the rows move
      c = Cand{nullptr, nullptr};
      if (hipMalloc((void**)&c.V, vb) != hipSuccess || hipMalloc((void**)&c.Vn, vb) != hipSuccess) {
        (void)hipGetLastError();  // no room for another trial: keep the best so far
        release(c);
        break;
      }
      if (hipMemcpyAsync(c.V, best.V, vb, hipMemcpyDeviceToDevice, e->stream) != hipSuccess) rc = GOSSIP_EHIP;
    }
    AeArgs d = make_ae_args(e);
    d.V = c.V;
    d.Vn = c.Vn;
    d.partial = part;
    d.aux = part + pl;
    d.zero = part;
    d.nzero = (uint32_t)(pl + 2);
    d.btl = e->ae_dg.tl;
    d.bnt = e->ae_dg.nt;
    d.boff = e->ae_dboff;
    d.dcap = e->ae_dcap;
    float ms = 0.f;
    for (int r = 0; r < 2 && rc == GOSSIP_OK; ++r) {
      if (r == 1 && hipEventRecord(ev[0], e->stream) != hipSuccess) rc = GOSSIP_EHIP;
      if (rc == GOSSIP_OK && launch_ae_dense_binned(d, e->stream) != hipSuccess) rc = GOSSIP_EHIP;
    }
    if (rc == GOSSIP_OK && (hipEventRecord(ev[1], e->stream) != hipSuccess ||
                            hipEventSynchronize(ev[1]) != hipSuccess ||
                            hipEventElapsedTime(&ms, ev[0], ev[1]) != hipSuccess))
      rc = GOSSIP_EHIP;
#ifdef GOSSIP_EXP_PLACE_LOG
    std::fprintf(stderr, "ae_place: candidate %u trial %.1f us\n", i, ms * 1e3);
#endif
    e->time_ms[5] += 2.0 * ms;
    e->launches[5] += 2;
    if (i == 0) {
      best_ms = ms;
      continue;
    }
    Cand loser = c;
    if (rc == GOSSIP_OK && ms < best_ms) {
      loser = best;
      best = c;
      best_ms = ms;
    }
    if (held.V) (void)hipStreamSynchronize(e->stream);  // (no trial is still reading the rows freed next)
    release(held);
    held = loser;
  }
  (void)hipEventDestroy(ev[0]);
  (void)hipEventDestroy(ev[1]);
  (void)hipFree(part);
  HIP_OK(e, hipStreamSynchronize(e->stream));
  release(held);
  e->V = best.V;  // (a candidate's V holds a copy of the rows)
  e->Vn = best.Vn;
  if (rc != GOSSIP_OK) return e->fail(rc, "ANTIENTROPY placement trial failed");
  return GOSSIP_OK;
}

int ae_round(gossip_engine* e) {
  int rc;
  bool sparse = ae_plan_sparse(e);
  if (!sparse && !e->ae_placed && (rc = ae_place(e))) return rc;
  e->ae_dense_next = false;
  e->ae_sparse_last = false;
  // partial and the aux words after it start at zero: cleared by the binned emit's block 0 (the
  // round's first kernel; no memset and no host gap, profiles/r05_ae3/), else by a memset
  const uint32_t nz = (uint32_t)(part_len(e) + 2);
  const bool dbin = e->ae_dbin && e->ae_dbin_on;
  if (sparse ? !e->ae_bin : !dbin) HIP_OK(e, hipMemsetAsync(e->partial_d, 0, (size_t)nz * 8, e->stream));
  if (sparse) {
    if (++e->ae_epoch == 0) {  // claims hold epochs: restart them after a wrap
      HIP_OK(e, hipMemsetAsync(e->ae_claim, 0, (size_t)e->N * 4, e->stream));
      e->ae_epoch = 1;
    }
    AeArgs a = make_ae_args(e);
    if ((rc = timer_begin(e, 2))) return rc;
    if (e->ae_bin) {
      a.zero = e->partial_d;
      a.nzero = nz;
      HIP_OK(e, launch_ae_sparse_binned(a, e->stream));  // churn fused into its first pass
      a.zero = nullptr;
    } else {
      HIP_OK(e, launch_ae_churn(a, e->stream));
      HIP_OK(e, launch_ae_sparse(a, e->stream));
    }
    if ((rc = timer_end(e, 2))) return rc;
    if ((rc = timer_begin(e, 1))) return rc;
    HIP_OK(e, launch_ae_sparse_stats(a, e->stream));
    if ((rc = timer_end(e, 1))) return rc;
    if ((rc = ae_read_back(e))) return rc;
    if (e->ae_aux_h[1] > e->ae_segcap) {  // overflow: only alive_n was written
      if ((rc = timer_collect(e))) return rc;
      ++e->ae_overflows;
      sparse = false;
      HIP_OK(e, hipMemsetAsync(e->partial_d, 0, (part_len(e) + 2) * 8, e->stream));  // partial and aux
    }
  }
  if (!sparse) {
    const AeArgs a = make_ae_args(e);
    bool binned = dbin;
    if (binned) {  // in-edge gathers, stats fused (no timer-1 part)
      AeArgs d = a;
      d.zero = e->partial_d;
      d.nzero = nz;
      d.btl = e->ae_dg.tl;
      d.bnt = e->ae_dg.nt;
      d.boff = e->ae_dboff;
      d.dcap = e->ae_dcap;
      // stale filter (param ae_dense_filter) once a tenth of the nodes is up to date: before that it
      // skips nothing and its checks cost
      if (e->ae_sb_valid && e->ae_dfilt && (double)e->ae_stale < 0.9 * (double)e->N) d.flags |= kAeSbValid;
      if ((rc = timer_begin(e, 0))) return rc;
      HIP_OK(e, launch_ae_dense_binned(d, e->stream));
      if ((rc = timer_end(e, 0))) return rc;
      if ((rc = ae_read_back(e))) return rc;
      if (e->ae_aux_h[1]) {  // a chunk's in-edges overflowed the LDS list: rerun with atomics
        if ((rc = timer_collect(e))) return rc;
        ++e->ae_dense_fallbacks;
        binned = false;
        HIP_OK(e, hipMemsetAsync(e->partial_d, 0, (part_len(e) + 2) * 8, e->stream));  // partial and aux
      }
    }
    if (!binned) {
      if ((rc = timer_begin(e, 0))) return rc;
      HIP_OK(e, launch_ae_churn(a, e->stream));
      HIP_OK(e, launch_ae_round(a, e->stream));
      if ((rc = timer_end(e, 0))) return rc;
      if ((rc = timer_begin(e, 1))) return rc;
      HIP_OK(e, launch_ae_stats(a, e->Vn, e->alive_n, true, e->stream));
      if ((rc = timer_end(e, 1))) return rc;
      if ((rc = ae_read_back(e))) return rc;
    }
  }
  // sparse rounds return the hash delta of the rows they changed
  e->ae_hash = sparse ? e->ae_hash + e->partial_h[3] : e->partial_h[3];
  e->ae_stale = e->ae_aux_h[0];
  e->ae_full = e->partial_h[0];
  e->ae_alive = e->partial_h[1];
  e->ae_sb_valid = true;
  e->ae_sparse_last = sparse;
  if (sparse) ++e->ae_sparse_rounds;
  return GOSSIP_OK;
}

// gossip_step of a one-engine ANTIENTROPY engine.  Dense rounds, and sparse
// rounds without the binned scan, run one at a time (ae_round: plan, kernels, totals read back).
// A run of sparse rounds is pipelined: up to ae_ahead rounds are enqueued at once, each with its
// own slot of totals and a gate word its emit writes from the previous round's slot (that round ran,
// its edge list did not overflow, it did not converge), so the sparse kernels of a round past convergence
// or after an overflow return at once; the host reads every slot after one sync.  An overflowed
// round left V, the bitmaps and the claims untouched: it is rerun dense (ae_dense_next), as
// ae_round does.  Every round's stats and state equal the unpipelined loop's; its path choice
// need not: the plan (ae_plan_sparse) is made once per batch, so a round the unpipelined loop
// would have planned dense (churn reviving stale nodes) may run sparse here, overflow and be
// rerun dense.  That moves ae_sparse_rounds, ae_overflows and timer 2, never a result bit.
int step_ae(gossip_engine* e, uint32_t max_rounds, gossip_round_stats_t* stats, uint64_t* infected,
            uint32_t* rounds_done) {
  const size_t pl = part_len(e), sw = pl + 2;  // a slot: the totals, then aux[0..1]
  if (!e->ae_slot_d) {
    HIP_OK(e, hipMalloc((void**)&e->ae_slot_d, kRing * sw * 8));
    HIP_OK(e, hipMalloc((void**)&e->ae_gate_d, kRing * 4));
    HIP_OK(e, hipHostMalloc((void**)&e->ae_slot_h, kRing * sw * 8, hipHostMallocDefault));
  }
  std::vector<uint64_t> part(pl);
  uint32_t r = 0;
  if (rounds_done) *rounds_done = 0;
  auto commit = [&](uint64_t* tot, bool* conv) -> int {  // one round's totals to the caller
    gossip_round_stats_t st;
    if (int rc = gossip_round_commit(e, tot, &st)) return rc;
    if (stats) stats[r] = st;
    if (infected) std::memcpy(infected + (size_t)r * e->R, tot + 4, (size_t)e->R * 8);
    ++r;
    if (rounds_done) *rounds_done = r;
    *conv = st.converged != 0;
    return GOSSIP_OK;
  };
  while (r < max_rounds) {
    bool conv = false;
    if (e->ae_ahead < 2 || !e->ae_bin || !ae_plan_sparse(e)) {  // one round, as the generic loop runs it
      if (int rc = gossip_round_compute(e, part.data())) return rc;
      if (int rc = commit(part.data(), &conv)) return rc;
      if (conv) break;
      continue;
    }
    const uint32_t A = std::min<uint32_t>(std::min<uint32_t>(e->ae_ahead, kRing), max_rounds - r);
    uint64_t *ab = e->alive, *abn = e->alive_n;
    for (uint32_t i = 0; i < A; ++i) {
      if (++e->ae_epoch == 0) {  // claims hold epochs: restart them after a wrap
        HIP_OK(e, hipMemsetAsync(e->ae_claim, 0, (size_t)e->N * 4, e->stream));
        e->ae_epoch = 1;
      }
      AeArgs a = make_ae_args(e);
      a.ab = ab;
      a.abn = abn;
      a.t = e->t + i;
      a.partial = e->ae_slot_d + i * sw;
      a.aux = a.partial + pl;
      // the emit opens or closes this round's gate from the previous round's slot and clears this
      // round's slot (no memset, no gate kernel per round: ~15 us each, profiles/r05_ae/)
      a.gate = e->ae_gate_d + i;
      a.gate_out = e->ae_gate_d + i;
      a.gate_prev = i ? e->ae_gate_d + (i - 1) : nullptr;
      a.prev_partial = i ? e->ae_slot_d + (i - 1) * sw : nullptr;
      a.pl = (uint32_t)pl;
      a.zero = a.partial;
      a.nzero = (uint32_t)sw;
      if (e->timing) HIP_OK(e, hipEventRecord(e->evr[i][0], e->stream));
      HIP_OK(e, launch_ae_sparse_binned(a, e->stream));  // churn fused into its first pass
      HIP_OK(e, launch_ae_sparse_stats(a, e->stream));
      if (e->timing) HIP_OK(e, hipEventRecord(e->evr[i][1], e->stream));
      std::swap(ab, abn);
    }
    HIP_OK(e, hipMemcpyAsync(e->ae_slot_h, e->ae_slot_d, A * sw * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(e, hipStreamSynchronize(e->stream));
    for (uint32_t i = 0; i < A; ++i) {  // round i ran: round i - 1 neither converged nor overflowed
      const uint64_t* tot = e->ae_slot_h + i * sw;
      const uint64_t* aux = tot + pl;
      if (aux[1] > e->ae_segcap) {  // overflow: the rounds after it did not run
        ++e->ae_overflows;
        e->ae_dense_next = true;
        break;
      }
      if (e->timing) {  // the whole sparse round (emit .. stats) in timer 2
        float ms = 0.f;
        HIP_OK(e, hipEventElapsedTime(&ms, e->evr[i][0], e->evr[i][1]));
        e->time_ms[2] += ms;
        e->launches[2] += 1;
      }
      // ae_round's bookkeeping of a sparse round, then gossip_round_compute's
      e->ae_hash += tot[3];
      e->ae_stale = aux[0];
      e->ae_full = tot[0];
      e->ae_alive = tot[1];
      e->ae_sb_valid = true;
      e->ae_sparse_last = true;
      ++e->ae_sparse_rounds;
      std::memcpy(part.data(), tot, pl * 8);
      part[3] = (e->cfg.flags & GOSSIP_FLAG_HASH) ? e->ae_hash : 0;
      e->last_sparse = false;
      if (int rc = commit(part.data(), &conv)) return rc;
      if (conv || r >= max_rounds) break;
    }
    if (conv) break;
  }
  return GOSSIP_OK;
}

// compute S_{t+1} of the owned shard from the gathered image + partial stats (device)
// A replicated dense round (plan kinds 5 / 6): the one-GPU binned round over the
// whole image of S_t (gathered by the driver for kind 5, left by the previous replicated round for
// kind 6) in place, so every rank holds S_{t+1} of every node; the rank reports the totals of its
// own slice (and rebuilds its own bitmaps) like any other sharded round, so the driver's
// all-reduce stays as it is.  Bits as the sharded kinds: the same draws and edges (§2).
int rep_compute(gossip_engine* e) {
  if (!e->rep_part) HIP_OK(e, hipMalloc((void**)&e->rep_part, (part_len(e) + 8) * 8));
  if (!e->rep_mem) {
    e->rbg = make_bin_geom(e->N, e->k, (e->N + kTileD - 1) / kTileD > kBigFromTiles);
    const size_t bytes = bin_bytes(e->rbg);
    if (hipMalloc(&e->rep_mem, bytes) != hipSuccess) {
      e->rep_mem = nullptr;
      return e->fail(GOSSIP_ENOMEM, "hipMalloc of %zu bytes (replicated-round records) failed", bytes);
    }
    const bool dyn = e->rbg.nt_d >= 4096;  // (the tile queues pay past 4096 tiles, as on one GPU)
    // placed as the one-GPU slab (place_bins): the trials read the image, write only records
    if (e->place_tries > 1 && bytes >= (512ull << 20)) {
      bool moved = false;
      if (int rc = place_slab(e, &e->rep_mem, bytes, [&](void* slab, float* ms) {
            return serve_trial(e, e->rbg, dyn, slab, current_image(e), e->rep_part, ms);
          }, &moved, "place_rep")) {
        (void)hipStreamSynchronize(e->stream);
        (void)hipFree(e->rep_mem);  // (never carved: the next replicated round allocates again)
        e->rep_mem = nullptr;
        return rc;
      }
    }
    bin_carve(e->rbg, e->rep_mem, &e->rbb);
    e->rbb.nzb = e->rbb.fullb = nullptr;  // (no edge filter: it needs bitmaps of the whole image)
    HIP_OK(e, hipMemset(e->rbb.dyn, 0, 17 * 4));
    if (!dyn) e->rbb.dyn = nullptr;
  }
  int rc;
  if ((rc = timer_begin(e, 0))) return rc;
  const RoundSync rs{nullptr, (uint32_t)part_len(e), 0u};
  HIP_OK(e, launch_binned_round(e->rbg, e->rbb, current_image(e), e->rep_part, e->R, e->t, e->key0, e->key1, e->mode,
                                0u, e->fa, e->cfg.flags, rs, e->stream));
  HIP_OK(e, hipMemsetAsync(e->partial_d, 0, part_len(e) * 8, e->stream));
  HIP_OK(e, launch_frontier_rebuild(e->lf, e->S, e->nown, e->partial_d, e->R, e->cfg.flags, e->stream));
  e->sx_valid = true;
  return timer_end(e, 0);
}

int compute_round(gossip_engine* e, const uint64_t* gathered) {
  const size_t bytes = (size_t)e->W * e->Nl * 8;
  if (e->mode == GOSSIP_MODE_ANTIENTROPY) return ae_round(e);  // (clears partial and aux itself)
  if (!e->binned) HIP_OK(e, hipMemsetAsync(e->partial_d, 0, part_len(e) * 8, e->stream));
  RoundArgs a = make_args(e, gathered);
  int rc;
  if (e->mode == GOSSIP_MODE_FLOOD) {
    if ((rc = timer_begin(e, 0))) return rc;
    if (e->flood_edges) {  // S_{t+1} starts as S_t; the walks OR deliveries into it
      HIP_OK(e, hipMemcpyAsync(e->Snext, e->S, bytes, hipMemcpyDeviceToDevice, e->stream));
      HIP_OK(e, launch_round_flood_walks(a, e->fw, e->stream));
    } else {
      HIP_OK(e, launch_round_flood(a, e->stream));
    }
    if ((rc = timer_end(e, 0))) return rc;
  } else if (e->binned) {  // one round, path chosen from the exact totals of S_t
    if ((rc = prepare_planned(e))) return rc;
    std::vector<uint64_t> tot;
    if ((rc = read_totals(e, &tot))) return rc;
    uint32_t maj = 0;
    bool all_d = false;
    const Est x = est_of(e, tot.data());
    const bool sparse = choose_sparse(e, x, &maj, &all_d);
    const uint32_t filt = dense_filter(e, x, filter_frac_of(e));
    if ((rc = timer_begin(e, 0))) return rc;
    if ((rc = launch_round_path(e, e->t, sparse, maj, all_d, filt,
                                ring_sync(e, 0), -1, sparse && bscan_round(e, x, maj))))
      return rc;
    return timer_end(e, 0);  // stats are fused into the round kernels
  } else if (e->rep_planned) {  // replicated dense round: the one-GPU round over the whole image
    return rep_compute(e);
  } else if (e->sbin) {  // sharded dense round: binned pipeline over the gathered image
    if ((rc = place_sb(e))) return rc;  // (a no-op once gossip_dense_prepare has placed the slab)
    if ((rc = timer_begin(e, 0))) return rc;
    if (e->sb_pre)  // the own-slice part was enqueued by gossip_dense_prepare
      HIP_OK(e, launch_sb_post(e->sbg, e->sbb, gathered, e->Snext, e->partial_d, e->R, e->t, e->key0, e->key1,
                               e->mode, e->fa, e->cfg.flags, e->lf.nzb, e->lf.fullb, e->stream));
    else
      HIP_OK(e, launch_sb_round(e->sbg, e->sbb, gathered, e->Snext, e->partial_d, e->R, e->t, e->key0, e->key1,
                                e->mode, e->fa, e->cfg.flags, e->lf.nzb, e->lf.fullb, e->stream));
    e->sb_pre = false;
    if ((rc = timer_end(e, 0))) return rc;
    e->sx_valid = true;  // totals of the own nodes and exact bitmaps of S_{t+1}, fused into the apply pass
    return GOSSIP_OK;
  } else {
    // timer 0 covers the whole S_t -> S_{t+1} transform (seed copy + round kernel)
    if ((rc = timer_begin(e, 0))) return rc;
    HIP_OK(e, hipMemcpyAsync(e->Snext, e->S, bytes, hipMemcpyDeviceToDevice, e->stream));
    HIP_OK(e, launch_round_random(a, e->stream));
    if ((rc = timer_end(e, 0))) return rc;
  }
  if ((rc = timer_begin(e, 1))) return rc;
  if (e->sx) {  // totals incl. nonzero nodes and exact bitmaps of S_{t+1}, for the next round's plan
    HIP_OK(e, launch_frontier_rebuild(e->lf, e->Snext, e->nown, e->partial_d, e->R, e->cfg.flags, e->stream));
    e->sx_valid = true;
  } else {
    HIP_OK(e, launch_stats(a, e->stream));
  }
  if ((rc = timer_end(e, 1))) return rc;
  return GOSSIP_OK;
}

void rotate(gossip_engine* e) {
  if (e->mode == GOSSIP_MODE_ANTIENTROPY) {
    if (!e->ae_sparse_last) std::swap(e->V, e->Vn);  // sparse rounds merge in place
    std::swap(e->alive, e->alive_n);
  } else if (e->mode == GOSSIP_MODE_FLOOD) {
    uint64_t* tmp = e->Sprev;
    e->Sprev = e->S;
    e->S = e->Snext;
    e->Snext = tmp;
  } else if (!e->binned) {  // binned rounds run in place
    e->cur ^= 1;
    bind_slices(e);
  }
}

AexArgs make_aex_args(gossip_engine* e) {
  AexArgs a{};
  a.V = e->V;
  a.Vn = e->Vn;
  a.img = e->aex_img;
  a.write_stale = true;
  a.target = e->target;
  a.partial = e->partial_d;
  a.cnt = e->aex_cnt;
  a.bcnt = e->aex_bcnt;
  a.boff = e->aex_boff;
  a.req = e->aex_req;
  a.loc = e->aex_loc;
  a.dirty = e->aex_track ? e->aex_dirty : nullptr;
  a.verdict = e->aex_verdict;
  a.N = e->N;
  a.Nl = e->Nl;
  a.lo = e->lo;
  a.nown = e->nown;
  a.G = e->G;
  a.rank = e->rank;
  a.K = e->R;
  a.L = ae_lanes(e->R);
  a.k = e->k;
  a.t = e->t;
  a.key0 = e->key0;
  a.key1 = e->key1;
  a.fail = e->cfg.churn_fail;
  a.rec = e->cfg.churn_recover;
  a.flags = e->cfg.flags;
  a.rw = e->aex_rw;
  a.pw = e->aex_pw;
  return a;
}

// ANTIENTROPY sparse-round edge lists.  cap_req = 0: the
// default capacity (N/8 edges covers the churn tail at configs[4]; small
// engines get room for every exchange, k per node, so never overflow); else
// exactly cap_req edges (gossip_set_param "ae_cap": the overflow tests).
int ae_alloc_lists(gossip_engine* e, uint64_t cap_req) {
  const uint64_t nw = (e->N + 63) / 64;
  const uint64_t kn = (uint64_t)e->N * e->k;
  const bool forced = cap_req != 0;
  const uint64_t cap = forced ? cap_req : std::min<uint64_t>(kn, std::max<uint64_t>(e->N / 8, 65536));
  if (e->ae_bin) {
    // binned scan: segment = peer tile.  A tile's segment holds every exchange on small
    // engines, else twice its share of the planned capacity (a larger segment overflows
    // and the round reruns dense)
    e->ae_nseg = e->ae_bg.nt;
    e->ae_spc = (uint32_t)((nw + e->ae_nseg - 1) / e->ae_nseg);
    e->ae_segcap = (cap >= kn && !forced) ? (uint32_t)kn : (uint32_t)((2 * cap + e->ae_nseg - 1) / e->ae_nseg);
    e->ae_cap = std::min<uint64_t>(cap, (uint64_t)e->ae_segcap * e->ae_nseg);
  } else {  // direct scan: block b owns ae_spc 64-node chunks and lists its edges in segment b
    e->ae_nseg = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(4096, (nw + 3) / 4));
    e->ae_spc = (uint32_t)((nw + e->ae_nseg - 1) / e->ae_nseg);
    e->ae_nseg = (uint32_t)((nw + e->ae_spc - 1) / e->ae_spc);
    e->ae_segcap = (cap >= kn && !forced) ? e->k * e->ae_spc * 64 : (uint32_t)((cap + e->ae_nseg - 1) / e->ae_nseg);
    e->ae_cap = (uint64_t)e->ae_segcap * e->ae_nseg;
  }
  void* old[] = {e->ae_segn, e->ae_eid, e->ae_erow};
  for (void* p : old)
    if (p) HIP_OK(e, hipFree(p));
  e->ae_segn = e->ae_eid = e->ae_erow = nullptr;
  const size_t seg_edges = (size_t)e->ae_segcap * e->ae_nseg;
  if (hipMalloc((void**)&e->ae_segn, (size_t)e->ae_nseg * 4) != hipSuccess ||
      hipMalloc((void**)&e->ae_eid, seg_edges * 8) != hipSuccess ||
      hipMalloc((void**)&e->ae_erow, seg_edges * 8 * e->R) != hipSuccess)
    return e->fail(GOSSIP_ENOMEM, "hipMalloc of the ANTIENTROPY edge lists (%llu edges) failed",
                   (unsigned long long)seg_edges);
  HIP_OK(e, hipMemset(e->ae_segn, 0, (size_t)e->ae_nseg * 4));
  return GOSSIP_OK;
}

void fill_stats(gossip_engine* e, const uint64_t* total, gossip_round_stats_t* st) {
  st->round = e->t;
  st->full_nodes = total[0];
  st->alive_nodes = total[1];
  st->converged = total[0] == total[1] ? 1u : 0u;
  st->messages = total[2];
  st->state_hash = (e->cfg.flags & GOSSIP_FLAG_HASH) ? total[3] : 0;
}

}  // namespace

extern "C" {

uint32_t gossip_abi_version(void) { return GOSSIP_ABI_VERSION; }

const char* gossip_last_error(const gossip_engine_t* eng) {
  return eng ? eng->err.c_str() : g_create_error.c_str();
}

int gossip_create(const gossip_config_t* cfg, gossip_engine_t** out) {
  g_create_error.clear();
  if (!cfg || !out) {
    g_create_error = "null argument";
    return GOSSIP_EINVAL;
  }
  *out = nullptr;
  if (cfg->n_nodes < 2 || cfg->n_nodes >= (1ull << 32)) {
    g_create_error = "n_nodes must be in [2, 2^32)";
    return GOSSIP_EINVAL;
  }
  if (cfg->n_rumors == 0 || cfg->n_rumors > 4096) {
    g_create_error = "n_rumors must be in [1, 4096]";
    return GOSSIP_EINVAL;
  }
  if (cfg->mode > GOSSIP_MODE_ANTIENTROPY) {
    g_create_error = "unknown mode";
    return GOSSIP_ENOTSUP;
  }
  if (cfg->mode == GOSSIP_MODE_ANTIENTROPY && cfg->n_rumors > 64) {
    g_create_error = "ANTIENTROPY has at most 64 components";
    return GOSSIP_ENOTSUP;
  }
  if (cfg->mode == GOSSIP_MODE_ANTIENTROPY && (cfg->shard_count ? cfg->shard_count : 1) > 1024) {
    g_create_error = "sharded ANTIENTROPY supports at most 1024 shards";
    return GOSSIP_ENOTSUP;
  }
  if (cfg->mode != GOSSIP_MODE_FLOOD && (cfg->fanout == 0 || cfg->fanout > 64)) {
    g_create_error = "fanout must be in [1, 64]";
    return GOSSIP_EINVAL;
  }
  const uint32_t G = cfg->shard_count ? cfg->shard_count : 1;
  if (cfg->shard_rank >= G) {
    g_create_error = "shard_rank >= shard_count";
    return GOSSIP_EINVAL;
  }
  if (cfg->stall_rounds > 16) {
    g_create_error = "stall_rounds must be in [0, 16]";
    return GOSSIP_EINVAL;
  }
  const bool faulty = cfg->edge_loss || cfg->partitions > 1 || cfg->stall_rounds;
  if (faulty && (cfg->mode == GOSSIP_MODE_ANTIENTROPY || (cfg->mode == GOSSIP_MODE_FLOOD && G != 1))) {
    g_create_error = "edge_loss / partitions / stall_rounds apply to the random modes and to one-shard FLOOD "
                     "(ANTIENTROPY's fault model is churn)";
    return GOSSIP_ENOTSUP;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    g_create_error = "no HIP device (libgossip_hip has no CPU fallback)";
    return GOSSIP_ENODEV;
  }
  int dev = cfg->device;
  if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (dev >= ndev) {
    g_create_error = "device ordinal out of range";
    return GOSSIP_ENODEV;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    g_create_error = std::string("device is not gfx950 (MI355X): ") + prop.gcnArchName;
    return GOSSIP_ENODEV;
  }

  gossip_engine* e = new gossip_engine();
  e->cfg = *cfg;
  e->device = dev;
  e->N = cfg->n_nodes;
  e->R = cfg->n_rumors;
  e->W = (e->R + 63) / 64;
  e->k = cfg->fanout;
  e->mode = cfg->mode;
  e->G = G;
  e->rank = cfg->shard_rank;
  e->Nl = (e->N + G - 1) / G;
  e->aex = e->mode == GOSSIP_MODE_ANTIENTROPY && G > 1;
  if (e->aex) e->Nl = (e->Nl + 63) / 64 * 64;  // 64-aligned row blocks: whole bitmap words per shard
  e->lo = std::min<uint64_t>((uint64_t)e->rank * e->Nl, e->N);
  e->hi = std::min<uint64_t>(e->lo + e->Nl, e->N);
  e->nown = e->hi - e->lo;
  e->key0 = (uint32_t)cfg->seed;
  e->key1 = (uint32_t)(cfg->seed >> 32);
  e->fa = Faults{cfg->edge_loss, cfg->partitions, cfg->n_nodes};
  e->timing = (cfg->flags & GOSSIP_FLAG_TIMING) != 0;
  e->flood_edges = e->mode == GOSSIP_MODE_FLOOD && faulty;
  e->fw.D = cfg->stall_rounds;

  auto bail = [&](int rc) {
    g_create_error = e->err;
    free_all(e);
    delete e;
    return rc;
  };
  if (hipSetDevice(dev) != hipSuccess) {
    e->err = "hipSetDevice failed";
    return bail(GOSSIP_EHIP);
  }
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
    e->err = "hipStreamCreate failed";
    return bail(GOSSIP_EHIP);
  }
  e->own_stream = true;
  const size_t shard = (size_t)e->W * e->Nl * 8;
  const size_t image = shard * G;
  auto alloc = [&](uint64_t** p, size_t bytes) {
    if (hipMalloc((void**)p, bytes) != hipSuccess) {
      e->err = "hipMalloc of " + std::to_string(bytes) + " bytes failed";
      return false;
    }
    return hipMemset(*p, 0, bytes) == hipSuccess;
  };
  if (!alloc(&e->partial_d, part_len(e) * 8 + 64) || !alloc(&e->scratch_d, 8)) return bail(GOSSIP_ENOMEM);
  if (cfg->stall_rounds && e->mode >= GOSSIP_MODE_PUSH && e->mode <= GOSSIP_MODE_PUSHPULL) {
    if (hipMalloc((void**)&e->stall_d, e->N) != hipSuccess || hipMemset(e->stall_d, 0, e->N) != hipSuccess) {
      e->err = "hipMalloc of the stall streaks failed";
      return bail(GOSSIP_ENOMEM);
    }
    e->fa.stall = e->stall_d;
    e->fa.D = cfg->stall_rounds;
  }
  if (e->flood_edges) {  // one walk per (value, node); none running until a value is injected or learned
    const size_t nw = (size_t)e->R * e->N;
    if (hipMalloc((void**)&e->fw.cur, nw * 4) != hipSuccess || hipMalloc((void**)&e->fw.snd, nw * 4) != hipSuccess ||
        hipMalloc((void**)&e->fw.att, nw) != hipSuccess || hipMemset(e->fw.cur, 0xFF, nw * 4) != hipSuccess ||
        hipMemset(e->fw.snd, 0xFF, nw * 4) != hipSuccess || hipMemset(e->fw.att, 0, nw) != hipSuccess) {
      e->err = "hipMalloc of the FLOOD walks failed";
      return bail(GOSSIP_ENOMEM);
    }
  }
  auto alloc_raw = [&](void** p, size_t bytes) {
    if (hipMalloc(p, bytes) != hipSuccess) {
      e->err = "hipMalloc of " + std::to_string(bytes) + " bytes failed";
      return false;
    }
    return hipMemset(*p, 0, bytes) == hipSuccess;
  };
  if (e->aex) {  // sharded ANTIENTROPY
    const size_t vb = std::max<size_t>((size_t)e->Nl * e->R * 4, 4);
    const size_t gw = (size_t)G * e->Nl / 64;  // bitmap words of all shards
    e->aex_rw = (e->R + 2 + 1) / 2 * 2;        // request item {p, n, row[K]}, padded to 8 B
    e->aex_pw = (e->R + 1) / 2 * 2;            // response item row[K], padded to 8 B
    e->aex_req_cap = std::max<uint64_t>(e->nown * e->k, 1);
    const size_t tab = aex_block_table_words(e->nown, G);
    if (!alloc_raw((void**)&e->V, vb) || !alloc_raw((void**)&e->Vn, vb) || !alloc_raw((void**)&e->target, 256) ||
        !alloc_raw((void**)&e->aex_img, gw * 16) || !alloc_raw((void**)&e->aex_cnt, (G + 1) * 8) ||
        !alloc_raw((void**)&e->aex_bcnt, tab * 4) || !alloc_raw((void**)&e->aex_boff, tab * 8) ||
        !alloc_raw((void**)&e->aex_req, e->aex_req_cap * e->aex_rw * 4) ||
        !alloc_raw((void**)&e->aex_loc, e->aex_req_cap * 8) ||
        !alloc_raw((void**)&e->aex_resp_in, e->aex_req_cap * e->aex_pw * 4) || !alloc_raw((void**)&e->aex_tmp, 256) ||
        !alloc_raw((void**)&e->aex_dirty, std::max<size_t>((e->Nl + 63) / 64, 1) * 8) ||
        !alloc_raw((void**)&e->aex_verdict, std::max<uint64_t>(e->nown, 1)))
      return bail(GOSSIP_ENOMEM);
    if (hipHostMalloc((void**)&e->aex_cnt_h, (G + 1) * 8) != hipSuccess) return bail(GOSSIP_ENOMEM);
    if (launch_aex_fill_alive(make_aex_args(e), nullptr) != hipSuccess) return bail(GOSSIP_EHIP);
  } else if (e->mode == GOSSIP_MODE_ANTIENTROPY) {
    const size_t vb = (size_t)e->N * e->R * 4;
    const size_t nw = ((size_t)e->N + 63) / 64;
    if (!alloc_raw((void**)&e->V, vb) || !alloc_raw((void**)&e->Vn, vb) || !alloc_raw((void**)&e->target, 256) ||
        !alloc_raw((void**)&e->alive, nw * 16) || !alloc_raw((void**)&e->alive_n, nw * 16))
      return bail(GOSSIP_ENOMEM);
    if (launch_ae_fill_alive(e->alive, e->N, nullptr) != hipSuccess) return bail(GOSSIP_EHIP);
    e->ae_bg = ae_bin_geom(e->N, e->k);
    e->ae_bin = !(cfg->flags & GOSSIP_FLAG_AE_DIRECT_SCAN) && e->k <= 16 && ae_bin_fits(e->ae_bg);  // else the direct scan
    e->ae_dg = ae_dense_geom(e->N, e->k);
    e->ae_dbin = ae_dense_fits(e->ae_dg, e->N, e->k, e->R);  // else pull + atomicMax push + stats
    if (e->ae_dbin && !alloc_raw((void**)&e->ae_dboff, (size_t)e->ae_dg.nreg * (e->ae_dg.nt + 1) * 2))
      return bail(GOSSIP_ENOMEM);
    if (e->ae_bin || e->ae_dbin) {
      const size_t recs = (size_t)e->ae_bg.nreg * ((size_t)e->k << e->ae_bg.rs);
      if (!alloc_raw((void**)&e->ae_brec, recs * 4) ||
          (e->ae_bin && !alloc_raw((void**)&e->ae_boff, (size_t)e->ae_bg.nreg * (e->ae_bg.nt + 1) * 2)))
        return bail(GOSSIP_ENOMEM);
    }
    e->ae_aux = e->partial_d + part_len(e);
    e->ae_aux_alias = true;
    if (!alloc_raw((void**)&e->ae_claim, (size_t)e->N * 4) ||
        !alloc_raw(&e->ae_pmask, (size_t)e->N * e->k * std::max<uint32_t>(1, ae_lanes(e->R) / 8)))
      return bail(GOSSIP_ENOMEM);
    if (ae_alloc_lists(e, 0) != GOSSIP_OK) return bail(GOSSIP_ENOMEM);
  } else if (e->mode == GOSSIP_MODE_FLOOD) {
    if (!alloc(&e->S, shard) || !alloc(&e->Snext, shard) || !alloc(&e->Sprev, shard) || !alloc(&e->skip, shard) ||
        !alloc(&e->imgF, image))
      return bail(GOSSIP_ENOMEM);
  } else if (!alloc(&e->img[0], image) || !alloc(&e->img[1], image)) {
    return bail(GOSSIP_ENOMEM);
  }
  bind_slices(e);
  if (e->mode != GOSSIP_MODE_FLOOD && e->mode != GOSSIP_MODE_ANTIENTROPY && !(cfg->flags & GOSSIP_FLAG_DIRECT) &&
      bin_path_ok(e->N, e->k, e->W, G)) {
    // past kBigFromTiles tiles the emit regions double (longer runs per tile, binned.hip V = 4, 5):
    // per dense round 2^25 nodes 1135 -> 1094 us, 2^26 2981 -> 2582 us; 2^24 slower (521 -> 583 us:
    // its runs of 16 records gain less than the big emit costs), profiles/r04_s
    e->bg = make_bin_geom(e->N, e->k, (e->N + kTileD - 1) / kTileD > kBigFromTiles);
    const size_t bytes = bin_bytes(e->bg);
    if (hipMalloc(&e->bin_mem, bytes) != hipSuccess) {
      e->err = "hipMalloc of " + std::to_string(bytes) + " bytes (bins) failed";
      return bail(GOSSIP_ENOMEM);
    }
    bin_carve(e->bg, e->bin_mem, &e->bb);
    // the serve / apply tile queues pay where a persistent block has many tiles: 2^27 nodes (32
    // per block) 5578 -> 5497 us per dense round; at 2^24 (4 per block) 510 -> 525 us
    // (profiles/r05_tq/); param tile_queues overrides
    e->bb_dyn = e->bb.dyn;
    if (hipMemset(e->bb_dyn, 0, 17 * 4) != hipSuccess) {  // (the first emit's queue; later rounds' transposes)
      e->err = "hipMemset of the tile queues failed";
      return bail(GOSSIP_EHIP);
    }
    if (e->bg.nt_d < 4096) e->bb.dyn = nullptr;
    e->binned = true;
    if (!(cfg->flags & GOSSIP_FLAG_DENSE)) {
      const size_t fbytes = frontier_bytes(e->N);
      if (!alloc_raw(&e->fr_mem, fbytes)) return bail(GOSSIP_ENOMEM);
      frontier_carve(e->N, e->fr_mem, &e->fb);
      e->bb.nzb = e->fb.nzb;
      e->bb.fullb = e->fb.fullb;
      e->frontier = true;
    }
    if (hipHostMalloc((void**)&e->ring_h, kRing * (part_len(e) + 1) * 8, hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void**)&e->ring_d, e->ring_h, 0) != hipSuccess) {
      e->err = "round ring allocation failed";
      return bail(GOSSIP_ENOMEM);
    }
    std::memset(e->ring_h, 0, kRing * (part_len(e) + 1) * 8);
  }
  if (G > 1 && G <= 1024 && e->W == 1 && e->mode >= GOSSIP_MODE_PUSH && e->mode <= GOSSIP_MODE_PUSHPULL &&
      !(cfg->flags & (GOSSIP_FLAG_DIRECT | GOSSIP_FLAG_DENSE))) {
    e->sg = SxGeom{e->N, e->Nl, e->lo, e->nown, G, e->rank, e->k, e->R};
    if (!alloc_raw(&e->lf_mem, frontier_bytes(e->nown)) || !alloc_raw(&e->sx_mem, sx_bytes(e->sg)))
      return bail(GOSSIP_ENOMEM);
    frontier_carve(e->nown, e->lf_mem, &e->lf);
    e->lf.id0 = e->lo;
    sx_carve(e->sg, e->sx_mem, &e->sb);
    if (hipHostMalloc((void**)&e->sx_host, (G + 2) * 8, hipHostMallocDefault) != hipSuccess) {
      e->err = "hipHostMalloc failed";
      return bail(GOSSIP_ENOMEM);
    }
    e->sx = true;
    if (!(cfg->flags & GOSSIP_FLAG_SHARD_DIRECT) && sb_path_ok(e->N, e->k, e->nown)) {
      e->sbg = make_sb_geom(e->N, e->k, e->lo, e->nown);
      if (!alloc_raw(&e->sb_mem, sb_bytes(e->sbg))) return bail(GOSSIP_ENOMEM);
      sb_carve(e->sbg, e->sb_mem, &e->sbb);
      e->sbin = true;
    }
    if (xd_path_ok(e->N, e->k, e->Nl, G)) {
      e->xg = make_xd_geom(e->N, e->k, e->Nl, e->lo, e->nown, G, e->rank);
      if (hipHostMalloc((void**)&e->xd_cnt_h, G * 4, hipHostMallocDefault) != hipSuccess) {
        e->err = "hipHostMalloc failed";
        return bail(GOSSIP_ENOMEM);
      }
      e->xd = true;
    }
    // sharded sparse rounds pay off up to a larger rare fraction than on one GPU: sparse_frac_of
  }
  if (hipHostMalloc((void**)&e->partial_h, part_len(e) * 8 + 64, hipHostMallocDefault) != hipSuccess) {
    e->err = "hipHostMalloc failed";
    return bail(GOSSIP_ENOMEM);
  }
  if (e->ae_aux_alias) e->ae_aux_h = e->partial_h + part_len(e);
  if (e->timing) {
    for (auto& p : e->ev)
      for (auto& x : p)
        if (hipEventCreate(&x) != hipSuccess) {
          e->err = "hipEventCreate failed";
          return bail(GOSSIP_EHIP);
        }
    for (auto& x : e->ev_pre)
      if (hipEventCreate(&x) != hipSuccess) {
        e->err = "hipEventCreate failed";
        return bail(GOSSIP_EHIP);
      }
    for (auto& p : e->evr)
      for (auto& x : p)
        if (hipEventCreate(&x) != hipSuccess) {
          e->err = "hipEventCreate failed";
          return bail(GOSSIP_EHIP);
        }
  }
  // the zeroing above ran on the null stream, which the engine's non-blocking
  // stream does not wait for: finish it before any engine work is enqueued
  if (hipDeviceSynchronize() != hipSuccess) {
    e->err = "hipDeviceSynchronize after allocation failed";
    return bail(GOSSIP_EHIP);
  }
  *out = e;
  return GOSSIP_OK;
}

void gossip_destroy(gossip_engine_t* eng) {
  if (!eng) return;
  (void)hipSetDevice(eng->device);
  (void)hipStreamSynchronize(eng->stream);  // (the null stream too, when bound)
  delete eng->tr;
  eng->tr = nullptr;
  (void)hipSetDevice(eng->device);
  free_all(eng);
  delete eng;
}

int gossip_set_stream(gossip_engine_t* e, void* hip_stream) {
  if (!e) return GOSSIP_EINVAL;
  if (int rc = set_dev(e)) return rc;
  if (!e->own_stream && e->stream == (hipStream_t)hip_stream) return GOSSIP_OK;
  HIP_OK(e, hipStreamSynchronize(e->stream));
  if (e->own_stream) HIP_OK(e, hipStreamDestroy(e->stream));
  // NULL is the legacy null stream (torch's default stream), not "keep my own":
  // a caller handing over its current stream is then ordered with its collectives
  e->stream = (hipStream_t)hip_stream;
  e->own_stream = false;
  return GOSSIP_OK;
}

int gossip_set_param(gossip_engine_t* e, const char* name, double v) {
  if (!e || !name) return GOSSIP_EINVAL;
  const std::string n(name);
  if (n == "sparse_frac") {
    e->sparse_frac = v;
    e->sparse_frac_set = true;
  } else if (n == "alld_frac") {
    e->alld_frac = v;
  } else if (n == "sparse_direct") {
    e->sparse_direct = v != 0;
  } else if (n == "ae_ahead") {
    if (v < 1 || v > kRing) return e->fail(GOSSIP_EINVAL, "ae_ahead: 1 .. %u", kRing);
    e->ae_ahead = (uint32_t)v;
  } else if (n == "ordered_collectives") {
    e->ordered = v != 0;
  } else if (n == "timing") {  // pause / resume the hipEvent timers of a GOSSIP_FLAG_TIMING engine
    if (v != 0 && v != 1) return e->fail(GOSSIP_EINVAL, "timing must be 0 or 1");
    if (v != 0 && !(e->cfg.flags & GOSSIP_FLAG_TIMING))
      return e->fail(GOSSIP_ESTATE, "timing needs an engine created with GOSSIP_FLAG_TIMING");
    if (int rc = timer_collect(e)) return rc;  // (no event of a timed round left pending)
    e->timing = v != 0;
  } else if (n == "place_tries") {
    if (v < 1 || v > 16) return e->fail(GOSSIP_EINVAL, "place_tries must be in [1, 16]");
    e->place_tries = (uint32_t)v;
  } else if (n == "link_gbps") {
    if (v < 0) return e->fail(GOSSIP_EINVAL, "link_gbps must be >= 0 (0 = fixed sparse_frac thresholds)");
    e->link_gbps = v;
  } else if (n == "rccl_dev_collectives") {
    e->rccl_dev = v != 0;
  } else if (n == "bin_scan_frac") {
    e->bscan_frac = v;
  } else if (n == "mid_frac") {
    e->mid_frac = v;
  } else if (n == "scan_queue") {
    e->fb.scan_q = e->lf.scan_q = v != 0 ? 1u : 0u;
  } else if (n == "filter_frac") {
    e->filter_frac = v;
    e->filter_frac_set = true;
  } else if (n == "xd_filter_frac") {
    e->xd_filter_frac = v;
  } else if (n == "ahead") {
    if (v < 1 || v > kRing - 1) return e->fail(GOSSIP_EINVAL, "ahead must be in [1, %u]", kRing - 1);
    e->ahead = (uint32_t)v;
  } else if (n == "replicate") {  // < 0: by the cost model, 0: never, > 0: every dense round
    e->replicate = v < 0 ? -1 : v > 0 ? 1 : 0;
  } else if (n == "cc_frac") {
    if (v < 0 || v > 1) return e->fail(GOSSIP_EINVAL, "cc_frac must be in [0, 1] (0 = never)");
    e->cc_frac = v;
  } else if (n == "xd_shards") {
    if (v < 0 || v > 1024) return e->fail(GOSSIP_EINVAL, "xd_shards must be in [0, 1024] (0 = never)");
    e->xd_shards = (uint32_t)v;
  } else if (n == "ae_sparse") {
    if (v != -1 && v != 0 && v != 1) return e->fail(GOSSIP_EINVAL, "ae_sparse must be -1, 0 or 1");
    e->ae_force = (int)v;
  } else if (n == "ae_dense_bin") {
    if (v != 0 && v != 1) return e->fail(GOSSIP_EINVAL, "ae_dense_bin must be 0 or 1");
    e->ae_dbin_on = v != 0;
  } else if (n == "ae_dense_filter") {
    e->ae_dfilt = v != 0;
  } else if (n == "ae_dense_cap") {
    if (v < 0 || v > 65535) return e->fail(GOSSIP_EINVAL, "ae_dense_cap must be in [0, 65535] (0 = default)");
    e->ae_dcap = (uint32_t)v;
  } else if (n == "ae_cap") {
    if (e->mode != GOSSIP_MODE_ANTIENTROPY) return e->fail(GOSSIP_ESTATE, "ae_cap needs ANTIENTROPY mode");
    if (e->aex) return e->fail(GOSSIP_ENOTSUP, "ae_cap: sharded ANTIENTROPY engines keep no edge lists");
    if (v < 0 || v > 4e9) return e->fail(GOSSIP_EINVAL, "ae_cap must be in [0, 4e9] (0 = default)");
    if (int rc = set_dev(e)) return rc;
    HIP_OK(e, hipStreamSynchronize(e->stream));
    return ae_alloc_lists(e, (uint64_t)v);
  } else {
    return e->fail(GOSSIP_EINVAL, "unknown parameter '%s'", name);
  }
  return GOSSIP_OK;
}

// "topology" handler (main.go:132-149).  Rows become sorted sets; the in-adjacency
// is built here once so the flood kernel can run as a race-free pull.
int gossip_set_topology_csr(gossip_engine_t* e, const uint32_t* row_ptr, const uint32_t* col, uint64_t n,
                            uint64_t n_edges) {
  if (!e || !row_ptr || (n_edges && !col)) return GOSSIP_EINVAL;
  if (n != e->N) return e->fail(GOSSIP_EINVAL, "topology has %llu nodes, engine has %llu",
                                (unsigned long long)n, (unsigned long long)e->N);
  if (row_ptr[0] != 0 || row_ptr[n] != n_edges) return e->fail(GOSSIP_EINVAL, "row_ptr does not span col");
  for (uint64_t u = 0; u < n; ++u)
    if (row_ptr[u + 1] < row_ptr[u]) return e->fail(GOSSIP_EINVAL, "row_ptr not monotone at %llu", (unsigned long long)u);
  for (uint64_t i = 0; i < n_edges; ++i)
    if (col[i] >= n) return e->fail(GOSSIP_EINVAL, "col[%llu] out of range", (unsigned long long)i);
  std::vector<uint32_t> orow(n + 1, 0), ocol;
  ocol.reserve(n_edges);
  for (uint64_t u = 0; u < n; ++u) {
    const size_t b = ocol.size();
    ocol.insert(ocol.end(), col + row_ptr[u], col + row_ptr[u + 1]);
    if (!e->flood_edges) {  // rows as sets; the walks of FLOOD with faults keep the message's list
      std::sort(ocol.begin() + b, ocol.end());
      ocol.erase(std::unique(ocol.begin() + b, ocol.end()), ocol.end());
    }
    orow[u + 1] = (uint32_t)ocol.size();
  }
  std::vector<uint32_t> irow(n + 1, 0), icol(ocol.size());
  for (uint32_t v : ocol) irow[v + 1]++;
  for (uint64_t v = 0; v < n; ++v) irow[v + 1] += irow[v];
  std::vector<uint32_t> fill(irow.begin(), irow.end() - 1);
  for (uint64_t u = 0; u < n; ++u)
    for (uint32_t q = orow[u]; q < orow[u + 1]; ++q) icol[fill[ocol[q]]++] = (uint32_t)u;
  if (int rc = set_dev(e)) return rc;
  HIP_OK(e, hipStreamSynchronize(e->stream));
  uint32_t** bufs[] = {&e->orow, &e->ocol, &e->irow, &e->icol};
  for (uint32_t** b : bufs)
    if (*b) {
      HIP_OK(e, hipFree(*b));
      *b = nullptr;
    }
  const size_t eb = std::max<size_t>(ocol.size(), 1) * 4, rb = (n + 1) * 4;
  if (hipMalloc((void**)&e->orow, rb) != hipSuccess || hipMalloc((void**)&e->ocol, eb) != hipSuccess ||
      hipMalloc((void**)&e->irow, rb) != hipSuccess || hipMalloc((void**)&e->icol, eb) != hipSuccess)
    return e->fail(GOSSIP_ENOMEM, "topology allocation failed");
  HIP_OK(e, hipMemcpy(e->orow, orow.data(), rb, hipMemcpyHostToDevice));
  HIP_OK(e, hipMemcpy(e->irow, irow.data(), rb, hipMemcpyHostToDevice));
  if (!ocol.empty()) {
    HIP_OK(e, hipMemcpy(e->ocol, ocol.data(), ocol.size() * 4, hipMemcpyHostToDevice));
    HIP_OK(e, hipMemcpy(e->icol, icol.data(), icol.size() * 4, hipMemcpyHostToDevice));
  }
  if (e->flood_edges) {  // a new topology ends every walk: the values held are not sent again
    const size_t nw = (size_t)e->R * e->N;
    HIP_OK(e, hipMemset(e->fw.cur, 0xFF, nw * 4));
    HIP_OK(e, hipMemset(e->fw.snd, 0xFF, nw * 4));
    HIP_OK(e, hipMemset(e->fw.att, 0, nw));
  }
  e->has_topo = true;
  return GOSSIP_OK;
}

int gossip_reset(gossip_engine_t* e) {
  if (!e) return GOSSIP_EINVAL;
  if (int rc = set_dev(e)) return rc;
  const size_t shard = (size_t)e->W * e->Nl * 8;
  if (e->aex) {
    HIP_OK(e, hipMemsetAsync(e->V, 0, (size_t)e->Nl * e->R * 4, e->stream));
    HIP_OK(e, hipMemsetAsync(e->target, 0, 256, e->stream));
    HIP_OK(e, launch_aex_fill_alive(make_aex_args(e), e->stream));
    e->aex_churned = ~0ull;
    e->aex_target_ok = e->aex_patch_ok = e->aex_inc_ok = false;
  } else if (e->mode == GOSSIP_MODE_ANTIENTROPY) {
    e->ae_v_zero = true;  // V: zeroed by the next call's set_dev, unless inject_random overwrites it
    HIP_OK(e, hipMemsetAsync(e->target, 0, 256, e->stream));
    HIP_OK(e, launch_ae_fill_alive(e->alive, e->N, e->stream));
    e->ae_sb_valid = false;
  } else if (e->mode == GOSSIP_MODE_FLOOD) {
    HIP_OK(e, hipMemsetAsync(e->S, 0, shard, e->stream));
    HIP_OK(e, hipMemsetAsync(e->Snext, 0, shard, e->stream));
    HIP_OK(e, hipMemsetAsync(e->Sprev, 0, shard, e->stream));
    HIP_OK(e, hipMemsetAsync(e->skip, 0, shard, e->stream));
    HIP_OK(e, hipMemsetAsync(e->imgF, 0, shard * e->G, e->stream));
  } else {
    // own slices only: every other slice of an image is written by the all-gather
    // before a round reads it, and a round writes the whole own slice of S_{t+1};
    // binned single-shard rounds run in place on S and never read the other image
    HIP_OK(e, hipMemsetAsync(e->S, 0, shard, e->stream));
    if (!e->binned) HIP_OK(e, hipMemsetAsync(e->Snext, 0, shard, e->stream));
  }
  if (e->stall_d) HIP_OK(e, hipMemsetAsync(e->stall_d, 0, e->N, e->stream));
  if (e->flood_edges) {
    const size_t nw = (size_t)e->R * e->N;
    HIP_OK(e, hipMemsetAsync(e->fw.cur, 0xFF, nw * 4, e->stream));
    HIP_OK(e, hipMemsetAsync(e->fw.snd, 0xFF, nw * 4, e->stream));
    HIP_OK(e, hipMemsetAsync(e->fw.att, 0, nw, e->stream));
  }
  e->fr_valid = false;
  e->sx_valid = e->gtot_valid = e->last_sparse = false;
  // a dense_prepare or sparse plan of the old state must not leak into the next round
  e->sb_pre = e->ev_pre_pending = e->sx_planned = e->xd_planned = e->cc_planned = false;
  e->rep_planned = e->rep_img_ok = false;
  if (e->frontier) {  // all-zero state: zero totals, empty bitmaps (D and its dirty flags are zero between rounds)
    const size_t nwb = (e->N + 63) / 64 * 8;
    HIP_OK(e, hipMemsetAsync(e->fb.nzb, 0, nwb, e->stream));
    HIP_OK(e, hipMemsetAsync(e->fb.fullb, 0, nwb, e->stream));
    HIP_OK(e, hipMemsetAsync(e->partial_d, 0, part_len(e) * 8, e->stream));
    e->fr_valid = true;
  }
  e->t = 0;
  return GOSSIP_OK;
}

int gossip_inject(gossip_engine_t* e, uint64_t node, uint32_t rumor) {
  if (!e) return GOSSIP_EINVAL;
  if (node >= e->N || rumor >= e->R) return e->fail(GOSSIP_EINVAL, "inject(%llu, %u) out of range",
                                                    (unsigned long long)node, rumor);
  if (int rc = set_dev(e)) return rc;
  if (e->aex) {  // a local write on the owner; the global max vector is re-derived before the next round
    if (node >= e->lo && node < e->hi)
      HIP_OK(e, launch_ae_inject(e->V, e->aex_tmp, node - e->lo, e->R, rumor, e->stream));
    e->aex_target_ok = e->aex_patch_ok = e->aex_inc_ok = false;
    return GOSSIP_OK;
  }
  if (e->mode == GOSSIP_MODE_ANTIENTROPY) {
    HIP_OK(e, launch_ae_inject(e->V, e->target, node, e->R, rumor, e->stream));
    e->ae_sb_valid = false;  // the target may have moved
    return GOSSIP_OK;
  }
  if (e->frontier && e->fr_valid) {
    HIP_OK(e, launch_frontier_inject(e->fb, e->S, e->N, e->partial_d, e->R, e->key0, e->key1, (int64_t)node, rumor,
                                     e->cfg.flags, e->stream));
    return GOSSIP_OK;
  }
  HIP_OK(e, launch_inject(e->S, e->Nl, e->lo, e->hi, e->N, e->R, e->key0, e->key1, (int64_t)node, rumor, e->stream,
                          e->flood_edges ? &e->fw : nullptr));
  e->fr_valid = e->sx_valid = e->gtot_valid = e->rep_img_ok = false;
  return GOSSIP_OK;
}

int gossip_inject_random(gossip_engine_t* e) {
  if (!e) return GOSSIP_EINVAL;
  if (e->mode == GOSSIP_MODE_ANTIENTROPY && !e->aex) e->ae_v_zero = false;  // ae_init writes every row
  if (int rc = set_dev(e)) return rc;
  if (e->aex) {
    HIP_OK(e, launch_aex_init(e->V, e->lo, e->nown, e->R, e->key0, e->key1, e->stream));
    e->aex_target_ok = e->aex_patch_ok = e->aex_inc_ok = false;
    return GOSSIP_OK;
  }
  if (e->mode == GOSSIP_MODE_ANTIENTROPY) {
    HIP_OK(e, launch_ae_init(e->V, e->target, e->N, e->R, e->key0, e->key1, e->stream));
    e->ae_sb_valid = false;
    return GOSSIP_OK;
  }
  if (e->frontier && e->fr_valid) {
    HIP_OK(e, launch_frontier_inject(e->fb, e->S, e->N, e->partial_d, e->R, e->key0, e->key1, -1, 0, e->cfg.flags,
                                     e->stream));
    return GOSSIP_OK;
  }
  HIP_OK(e, launch_inject(e->S, e->Nl, e->lo, e->hi, e->N, e->R, e->key0, e->key1, -1, 0, e->stream,
                          e->flood_edges ? &e->fw : nullptr));
  e->fr_valid = e->sx_valid = e->gtot_valid = e->rep_img_ok = false;
  return GOSSIP_OK;
}

uint64_t gossip_partial_len(const gossip_engine_t* e) { return e ? part_len(e) : 0; }

int gossip_exchange_buffers(gossip_engine_t* e, void** send, void** recv, uint64_t* send_bytes) {
  if (!e) return GOSSIP_EINVAL;
  if (e->mode == GOSSIP_MODE_FLOOD && !e->has_topo) return e->fail(GOSSIP_ESTATE, "FLOOD needs a topology");
  if (int rc = set_dev(e)) return rc;
  // the state all-gather rounds' slab is placed before the first collective starts: trials
  // timed while the all-gather runs would read a half-written image under link traffic (a
  // replicated round does not use it)
  if (!e->rep_planned)
    if (int rc = place_sb(e)) return rc;
  uint64_t *s = nullptr, *img = nullptr;
  if (int rc = prepare_send(e, &s, &img)) return rc;
  // the caller's collective runs on another stream: publish the slice first
  if (!e->driven && !e->ordered) HIP_OK(e, hipStreamSynchronize(e->stream));
  if (send) *send = s;
  if (recv) *recv = img;
  if (send_bytes) *send_bytes = e->aex ? e->Nl / 4 : (uint64_t)e->W * e->Nl * 8;
  return GOSSIP_OK;
}

int gossip_dense_prepare(gossip_engine_t* e) {
  if (!e) return GOSSIP_EINVAL;
  if (!e->sbin || e->sb_pre || e->rep_planned) return GOSSIP_OK;
  if (int rc = set_dev(e)) return rc;
  if (int rc = place_sb(e)) return rc;  // (placed already by gossip_exchange_buffers / gossip_cc_send)
  if (e->timing) HIP_OK(e, hipEventRecord(e->ev_pre[0], e->stream));
  HIP_OK(e, launch_sb_pre(e->sbg, e->sbb, current_image(e), e->R, e->t, e->key0, e->key1, e->mode, e->fa,
                          e->stream));
  if (e->timing) {
    HIP_OK(e, hipEventRecord(e->ev_pre[1], e->stream));
    e->ev_pre_pending = true;
  }
  e->sb_pre = true;
  return GOSSIP_OK;
}

namespace {
// --- device values for device-side collectives (the gossip_*_dev calls) ---
// pub_d: [0, G) per-rank counts, [G] one count, [G + 2, G + 2 + part_len) partials.
int pub_alloc(gossip_engine* e) {
  if (e->pub_d) return GOSSIP_OK;
  HIP_OK(e, hipMalloc((void**)&e->pub_d, (e->G + 2 + part_len(e)) * 8));
  return GOSSIP_OK;
}
uint64_t* pub_counts(gossip_engine* e) { return e->pub_d; }
uint64_t* pub_count(gossip_engine* e) { return e->pub_d + e->G; }
uint64_t* pub_partial(gossip_engine* e) { return e->pub_d + e->G + 2; }
// the own partials with the node count in slot 1 (what copy_partial_out hands the host)
int pub_partial_out(gossip_engine* e) {
  HIP_OK(e, launch_publish(e->partial_d, nullptr, pub_partial(e), (uint32_t)part_len(e), 1, e->nown, e->stream));
  return GOSSIP_OK;
}
// A published value is ready for work enqueued later on the engine's stream; a caller whose
// collectives run elsewhere gets it after a sync.  Timing (probe) mode syncs and folds the timers.
int pub_ready(gossip_engine* e, bool collect, bool count = true) {
  if (e->timing || (!e->driven && !e->ordered)) HIP_OK(e, hipStreamSynchronize(e->stream));
  if (e->timing && collect) return timer_collect(e, count);
  return GOSSIP_OK;
}
}  // namespace

int gossip_round_compute(gossip_engine_t* e, uint64_t* partial) {
  if (!e || !partial) return GOSSIP_EINVAL;
  if (e->aex) return e->fail(GOSSIP_ESTATE, "sharded ANTIENTROPY rounds run through the gossip_ae_* calls");
  if (e->mode == GOSSIP_MODE_FLOOD && !e->has_topo) return e->fail(GOSSIP_ESTATE, "FLOOD needs a topology");
  if (int rc = set_dev(e)) return rc;
  if (int rc = compute_round(e, current_image(e))) return rc;
  if (e->mode != GOSSIP_MODE_ANTIENTROPY) {  // (ae_round read partial and aux back already)
    HIP_OK(e, hipMemcpyAsync(e->partial_h, e->partial_d, part_len(e) * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(e, hipStreamSynchronize(e->stream));
  }
  if (int rc = timer_collect(e)) return rc;
  std::memcpy(partial, e->partial_h, part_len(e) * 8);
  if (e->mode != GOSSIP_MODE_ANTIENTROPY) partial[1] = e->nown;
  else partial[3] = (e->cfg.flags & GOSSIP_FLAG_HASH) ? e->ae_hash : 0;
  e->last_sparse = false;
  return GOSSIP_OK;
}

int gossip_round_compute_dev(gossip_engine_t* e, const uint64_t** partial) {
  if (!e || !partial) return GOSSIP_EINVAL;
  if (e->aex || e->mode == GOSSIP_MODE_ANTIENTROPY)
    return e->fail(GOSSIP_ENOTSUP, "ANTIENTROPY partials are finished on the host: gossip_round_compute");
  if (e->mode == GOSSIP_MODE_FLOOD && !e->has_topo) return e->fail(GOSSIP_ESTATE, "FLOOD needs a topology");
  if (int rc = set_dev(e)) return rc;
  if (int rc = pub_alloc(e)) return rc;
  if (int rc = compute_round(e, current_image(e))) return rc;
  if (int rc = pub_partial_out(e)) return rc;
  if (int rc = pub_ready(e, true)) return rc;
  e->last_sparse = false;
  *partial = pub_partial(e);
  return GOSSIP_OK;
}

int gossip_round_commit(gossip_engine_t* e, const uint64_t* total, gossip_round_stats_t* st) {
  if (!e || !total) return GOSSIP_EINVAL;
  if (e->stall_d) {  // stall streaks after round t, every shard over all N nodes
    if (int rc = set_dev(e)) return rc;
    HIP_OK(e, launch_stall_update(e->stall_d, e->N, e->k, e->t, e->key0, e->key1, e->fa, e->stream));
  }
  if (!e->last_sparse && !e->rep_planned) rotate(e);  // sparse and replicated rounds update S in place
  e->rep_img_ok = e->rep_planned;  // a replicated round leaves S_{t+1} of every node in the image
  e->rep_planned = false;
  if (e->aex) {  // V = S_{t+1}, Vn = S_t, aex_dirty = the rows where they differ
    e->aex_patch_ok = e->aex_round_done;
    e->aex_round_done = false;
  }
  e->last_sparse = false;
  if (e->sx) {  // global totals of S_{t+1}: the next round's plan
    e->gtot.assign(total, total + part_len(e));
    e->gtot_valid = true;
  }
  if (st) fill_stats(e, total, st);
  e->t++;
  return GOSSIP_OK;
}

// --- sharded sparse rounds (sharded.h) ---------------------------------------

namespace {

// exact totals of the owned nodes in partial_d and exact bitmaps in lf
int sx_prepare(gossip_engine* e) {
  if (e->sx_valid) return GOSSIP_OK;
  HIP_OK(e, hipMemsetAsync(e->partial_d, 0, part_len(e) * 8, e->stream));
  HIP_OK(e, launch_frontier_rebuild(e->lf, e->S, e->nown, e->partial_d, e->R, e->cfg.flags, e->stream));
  e->sx_valid = true;
  return GOSSIP_OK;
}

int sx_check(gossip_engine* e, bool planned) {
  if (!e) return GOSSIP_EINVAL;
  if (!e->sx) return e->fail(GOSSIP_ENOTSUP, "sparse sharded rounds need G > 1, W == 1 and a random mode");
  if (planned && !e->sx_planned) return e->fail(GOSSIP_ESTATE, "gossip_sharded_plan did not plan a sparse round");
  return set_dev(e);
}

int grow(gossip_engine* e, SxItem** buf, uint64_t* cap, uint64_t items) {
  if (items <= *cap && *buf) return GOSSIP_OK;
  const uint64_t want = std::max<uint64_t>(items + items / 4, 1024);
  if (*buf) HIP_OK(e, hipFree(*buf));
  *buf = nullptr;
  *cap = 0;
  HIP_OK(e, hipMalloc((void**)buf, want * sizeof(SxItem)));
  *cap = want;
  return GOSSIP_OK;
}

int copy_partial_out(gossip_engine* e, uint64_t* partial) {
  HIP_OK(e, hipMemcpyAsync(e->partial_h, e->partial_d, part_len(e) * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  std::memcpy(partial, e->partial_h, part_len(e) * 8);
  partial[1] = e->nown;
  return GOSSIP_OK;
}

}  // namespace

int gossip_local_totals(gossip_engine_t* e, uint64_t* partial) {
  if (!partial) return GOSSIP_EINVAL;
  if (int rc = sx_check(e, false)) return rc;
  if (int rc = sx_prepare(e)) return rc;
  return copy_partial_out(e, partial);
}

int gossip_sharded_plan(gossip_engine_t* e, const uint64_t* total, int32_t* kind) {
  if (!e || !kind) return GOSSIP_EINVAL;
  e->sx_planned = e->xd_planned = e->cc_planned = e->rep_planned = false;
  if (e->aex) {  // 2: an anti-entropy exchange round; -2: the global max vector is needed first
    *kind = e->aex_target_ok ? 2 : -2;
    return GOSSIP_OK;
  }
  if (!e->sx) {
    *kind = 0;
    return GOSSIP_OK;
  }
  if (total) {
    e->gtot.assign(total, total + part_len(e));
    e->gtot_valid = true;
  }
  if (!e->gtot_valid) {
    *kind = -1;
    return GOSSIP_OK;
  }
  uint32_t maj = 0;
  bool all_d = false;
  e->sx_planned = choose_sparse(e, est_of(e, e->gtot.data()), &maj, &all_d);
  // (link_gbps 0: priced at the default rate, for gossip_plan_model only)
  const ShardCosts c = shard_round_costs(e, est_of(e, e->gtot.data()));
  const bool model = !e->sparse_frac_set && e->link_gbps > 0;
  // replicated dense rounds: forced (param replicate 1), or by the model: with a whole image
  // (kind 6) while one costs less than the sharded dense round; entering (kind 5: the all-gather
  // plus the whole round) where what it costs over the sharded round is won back over the dense
  // rounds the mean-field predictor (§3.4) sees ahead.  The model's per-node fits come from
  // 2^24-2^27-node runs: below 2^22 nodes it replicates only when forced
  const double rep6 = c.rep - c.rep_link;
  bool rep_auto = e->replicate < 0 && model && e->N >= (1ull << 22) && rep6 < c.dense;
  if (rep_auto && !e->rep_img_ok) rep_auto = c.rep - c.dense < rep_gain_ahead(e, est_of(e, e->gtot.data()));
  const bool rep_any = c.rep_ok && (e->replicate == 1 || rep_auto);
  if (model)  // the link-aware cost model decides instead
    e->sx_planned = c.sparse < (rep_any ? std::min(c.dense, c.rep) : c.dense);
  e->rep_planned = !e->sx_planned && rep_any;
  e->plan_cost[0] = c.sparse;
  e->plan_cost[1] = c.dense;
  e->sx_maj = maj;
  e->sx_alld = all_d;
  {  // the mid-level summary of the global rare bitmap (choose_sparse's rule, sharded summary)
    const Est x = est_of(e, e->gtot.data());
    const double r = std::min(1.0, std::min(x.nz, (double)e->N - x.full) / (double)e->N);
    e->sx_mid = e->sb.gsum.summ2 && 1.0 - std::pow(1.0 - r, (double)(1u << e->sb.gsum.glog)) >= e->mid_frac;
  }
  e->xd_planned = !e->sx_planned && !e->rep_planned && e->xd && e->xd_shards && e->G >= e->xd_shards;
  // exchange rounds drop the one-way edges into empty / full peers when many nodes are (the
  // global totals are exact: no prediction), after an all-gather of the class bitmaps
  // (k <= 8: one keep byte per sender carries the count pass's probes to the emit pass)
  e->xd_filt = e->xd_planned && e->k <= 8 ? dense_filter(e, est_of(e, e->gtot.data()), e->xd_filter_frac) : 0u;
  e->xd_cls_ok = false;
  // dense on the state image: class-coded when few nodes are mixed (neither empty nor full)
  const double mixed = ((double)e->gtot[4 + e->R] - (double)e->gtot[0]) / (double)e->N;
  // entering replication over the class-coded all-gather (kind 7): the image expanded whole, then
  // the replicated round
  const bool rep_cc = e->rep_planned && !e->rep_img_ok && c.dense_cc;
  e->cc_planned = (!e->sx_planned && !e->xd_planned && !e->rep_planned && e->cc_frac > 0 && mixed <= e->cc_frac) || rep_cc;
  *kind = e->sx_planned ? 1 : e->rep_planned ? (e->rep_img_ok ? 6 : rep_cc ? 7 : 5) : e->xd_planned ? 3 : e->cc_planned ? 4 : 0;
  // the model's price of the round as planned (gossip_plan_model): the plan of the current run
  // (restarted at round 0) and the modelled ms since gossip_reset_timing
  if (e->t == 0) e->model_plan.clear();
  e->model_plan.push_back("DSAXCRrQ"[*kind]);
  e->model_ms += e->sx_planned ? c.sparse : e->rep_planned ? c.rep : c.dense;
  e->model_link_ms += e->sx_planned ? c.sparse_link : e->rep_planned ? c.rep_link : c.dense_link;
  e->model_rounds += 1;
  return GOSSIP_OK;
}

int gossip_sparse_rare(gossip_engine_t* e, void** send, uint64_t* count) {
  if (!send || !count) return GOSSIP_EINVAL;
  if (int rc = sx_check(e, true)) return rc;
  if (int rc = sx_prepare(e)) return rc;
  HIP_OK(e, sx_compact(e->sg, e->sb, e->lf, e->S, e->sx_maj, e->stream));
  const uint64_t nwl = (e->nown + 63) / 64;  // (the count: the word after the per-word bases)
  e->sx_host[0] = 0;
  HIP_OK(e, hipMemcpyAsync(e->sx_host, e->sb.wpos + nwl, 4, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  *count = e->sx_host[0] & 0xFFFFFFFFull;
  *send = e->sb.rare_send;
  return GOSSIP_OK;
}

int gossip_sparse_rare_dev(gossip_engine_t* e, void** send, const uint64_t** count) {
  if (!send || !count) return GOSSIP_EINVAL;
  if (int rc = sx_check(e, true)) return rc;
  if (int rc = pub_alloc(e)) return rc;
  if (int rc = sx_prepare(e)) return rc;
  HIP_OK(e, sx_compact(e->sg, e->sb, e->lf, e->S, e->sx_maj, e->stream));
  const uint64_t nwl = (e->nown + 63) / 64;
  HIP_OK(e, launch_publish(nullptr, e->sb.wpos + nwl, pub_count(e), 1, -1, 0, e->stream));
  if (int rc = pub_ready(e, false)) return rc;
  *count = pub_count(e);
  *send = e->sb.rare_send;
  return GOSSIP_OK;
}

int gossip_sparse_rare_recv(gossip_engine_t* e, uint64_t stride, void** recv) {
  if (!recv) return GOSSIP_EINVAL;
  if (int rc = sx_check(e, true)) return rc;
  if (stride > e->Nl) return e->fail(GOSSIP_EINVAL, "rare list stride %llu > nodes per shard", (unsigned long long)stride);
  if (int rc = grow(e, &e->rare_recv, &e->rare_recv_cap, stride * e->G)) return rc;
  e->sx_stride = stride;
  *recv = e->rare_recv;
  return GOSSIP_OK;
}

namespace {
// the rare lists' bases, the index and the scan (the per-owner counts land in sb.msg_cnt)
int sparse_scan_enqueue(gossip_engine* e, const uint64_t* counts) {
  if (!e->rare_recv) return e->fail(GOSSIP_ESTATE, "gossip_sparse_rare_recv first");
  uint64_t* cb = e->sx_host;
  cb[0] = 0;
  for (uint32_t q = 0; q < e->G; ++q) {
    if (counts[q] > e->sx_stride) return e->fail(GOSSIP_EINVAL, "rare list %u longer than the stride", q);
    cb[q + 1] = cb[q] + counts[q];
  }
  HIP_OK(e, hipMemcpyAsync(e->sb.cbase, cb, (e->G + 1) * 8, hipMemcpyHostToDevice, e->stream));
  if (int rc = timer_begin(e, 0)) return rc;
  const uint64_t rare = cb[e->G];
  HIP_OK(e, sx_index(e->sg, e->sb, e->rare_recv, e->sx_stride, rare, e->stream, e->sx_mid));
  HIP_OK(e, sx_scan(e->sg, e->sb, e->lf, e->S, e->rare_recv, e->sx_stride, rare, e->t, e->key0, e->key1, e->mode,
                    e->sx_maj, e->sx_alld, e->fa, e->stream, e->sx_mid));
  return timer_end(e, 0);
}
}  // namespace

int gossip_sparse_scan(gossip_engine_t* e, const uint64_t* counts, void** send, uint64_t* send_counts) {
  if (!counts || !send || !send_counts) return GOSSIP_EINVAL;
  if (int rc = sx_check(e, true)) return rc;
  if (int rc = sparse_scan_enqueue(e, counts)) return rc;
  // (the copy below lands in cb's pinned buffer after the copy that read it: same stream)
  HIP_OK(e, hipMemcpyAsync(e->sx_host, e->sb.msg_cnt, (e->G + 1) * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  const uint32_t* c = (const uint32_t*)e->sx_host;
  for (uint32_t q = 0; q < e->G; ++q) send_counts[q] = c[q];
  *send = e->sb.msg_out;
  return GOSSIP_OK;
}

int gossip_sparse_scan_dev(gossip_engine_t* e, const uint64_t* counts, void** send, const uint64_t** send_counts) {
  if (!counts || !send || !send_counts) return GOSSIP_EINVAL;
  if (int rc = sx_check(e, true)) return rc;
  if (int rc = pub_alloc(e)) return rc;
  // (the bases' host-to-device copy reads sx_host: the caller's next host read of a device value
  // syncs the stream before sx_host is written again)
  if (int rc = sparse_scan_enqueue(e, counts)) return rc;
  HIP_OK(e, launch_publish(nullptr, e->sb.msg_cnt, pub_counts(e), e->G, -1, 0, e->stream));
  if (int rc = pub_ready(e, false)) return rc;
  *send_counts = pub_counts(e);
  *send = e->sb.msg_out;
  return GOSSIP_OK;
}

int gossip_sparse_msg_recv(gossip_engine_t* e, uint64_t items, void** recv) {
  if (!recv) return GOSSIP_EINVAL;
  if (int rc = sx_check(e, true)) return rc;
  if (int rc = grow(e, &e->msg_recv, &e->msg_recv_cap, items)) return rc;
  *recv = e->msg_recv;
  return GOSSIP_OK;
}

namespace {
int sparse_commit_enqueue(gossip_engine* e, uint64_t items) {
  if (items > e->msg_recv_cap) return e->fail(GOSSIP_EINVAL, "more messages than the receive buffer holds");
  if (int rc = timer_begin(e, 1)) return rc;
  HIP_OK(e, sx_apply(e->lf, e->msg_recv, items, e->sx_alld, e->stream));
  HIP_OK(e, launch_frontier_commit(e->lf, e->S, e->nown, e->partial_d, e->R, e->sx_alld ? kSparseAllD : kSparseFlags,
                                   e->cfg.flags, e->stream));
  return timer_end(e, 1);
}
}  // namespace

int gossip_sparse_commit(gossip_engine_t* e, uint64_t items, uint64_t* partial) {
  if (!partial) return GOSSIP_EINVAL;
  if (int rc = sx_check(e, true)) return rc;
  if (int rc = sparse_commit_enqueue(e, items)) return rc;
  if (int rc = copy_partial_out(e, partial)) return rc;
  if (int rc = timer_collect(e)) return rc;
  e->sx_planned = false;
  e->last_sparse = true;
  return GOSSIP_OK;
}

int gossip_sparse_commit_dev(gossip_engine_t* e, uint64_t items, const uint64_t** partial) {
  if (!partial) return GOSSIP_EINVAL;
  if (int rc = sx_check(e, true)) return rc;
  if (int rc = pub_alloc(e)) return rc;
  if (int rc = sparse_commit_enqueue(e, items)) return rc;
  if (int rc = pub_partial_out(e)) return rc;
  if (int rc = pub_ready(e, true)) return rc;
  e->sx_planned = false;
  e->last_sparse = true;
  *partial = pub_partial(e);
  return GOSSIP_OK;
}

// --- class-coded state exchange (include/gossip.h gossip_cc_*) --------

namespace {
int cc_check(gossip_engine* e) {
  if (!e) return GOSSIP_EINVAL;
  if (!e->cc_planned) return e->fail(GOSSIP_ESTATE, "gossip_sharded_plan did not plan a class-coded round");
  return set_dev(e);
}
}  // namespace

int gossip_cc_send(gossip_engine_t* e, void** bits, uint64_t* bits_bytes, void** vals, uint64_t* count) {
  if (!bits || !bits_bytes || !vals || !count) return GOSSIP_EINVAL;
  if (int rc = cc_check(e)) return rc;
  if (!e->rep_planned)  // (as in gossip_exchange_buffers: before the collectives)
    if (int rc = place_sb(e)) return rc;
  const uint64_t nwl = (e->Nl + 63) / 64, slot = cc_slot_words(e->Nl);
  if (!e->cc_bits) {
    HIP_OK(e, hipMalloc((void**)&e->cc_bits, (size_t)e->G * slot * 8));
    HIP_OK(e, hipMemsetAsync(e->cc_bits, 0, (size_t)e->G * slot * 8, e->stream));
  }
  if (int rc = sx_prepare(e)) return rc;  // exact occupancy bitmaps of S_t
  uint64_t* out = (uint64_t*)e->sb.rare_send;  // Nl 16-B items of room: Nl words here
  HIP_OK(e, cc_compact(e->sg, e->sb, e->lf, e->S, out, e->stream));
  uint64_t* own = e->cc_bits + (size_t)e->rank * slot;
  const uint64_t nwo = (e->nown + 63) / 64;  // (a short last shard: its tail words stay zero)
  HIP_OK(e, hipMemcpyAsync(own, e->lf.nzb, nwo * 8, hipMemcpyDeviceToDevice, e->stream));
  HIP_OK(e, hipMemcpyAsync(own + nwl, e->lf.fullb, nwo * 8, hipMemcpyDeviceToDevice, e->stream));
  HIP_OK(e, hipMemcpyAsync(own + 2 * nwl, e->sb.wpos, nwo * 4, hipMemcpyDeviceToDevice, e->stream));
  e->sx_host[0] = 0;
  HIP_OK(e, hipMemcpyAsync(e->sx_host, e->sb.wpos + nwo, 4, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  *count = e->sx_host[0] & 0xFFFFFFFFull;
  *bits = own;
  *bits_bytes = slot * 8;
  *vals = out;
  return GOSSIP_OK;
}

int gossip_cc_recv(gossip_engine_t* e, uint64_t stride, void** bits_image, void** vals) {
  if (!bits_image || !vals) return GOSSIP_EINVAL;
  if (int rc = cc_check(e)) return rc;
  if (!e->cc_bits) return e->fail(GOSSIP_ESTATE, "gossip_cc_send first");
  if (stride > e->Nl) return e->fail(GOSSIP_EINVAL, "stride %llu > nodes per shard", (unsigned long long)stride);
  const uint64_t want = std::max<uint64_t>(stride * e->G, 1);
  if (want > e->cc_vals_cap) {
    HIP_OK(e, hipStreamSynchronize(e->stream));
    if (e->cc_vals) HIP_OK(e, hipFree(e->cc_vals));
    e->cc_vals = nullptr;
    e->cc_vals_cap = 0;
    const uint64_t cap = want + want / 4;
    HIP_OK(e, hipMalloc((void**)&e->cc_vals, cap * 8));
    e->cc_vals_cap = cap;
  }
  e->cc_stride = stride;
  *bits_image = e->cc_bits;
  *vals = e->cc_vals;
  return GOSSIP_OK;
}

int gossip_cc_expand(gossip_engine_t* e, const uint64_t* counts) {
  if (!counts) return GOSSIP_EINVAL;
  if (int rc = cc_check(e)) return rc;
  if (!e->cc_vals) return e->fail(GOSSIP_ESTATE, "gossip_cc_recv first");
  for (uint32_t q = 0; q < e->G; ++q)
    if (counts[q] > e->cc_stride) return e->fail(GOSSIP_EINVAL, "shard %u sent more mixed words than the stride", q);
  HIP_OK(e, cc_expand(e->sg, e->cc_bits, e->cc_vals, e->cc_stride, current_image(e), e->R, e->stream));
  e->cc_planned = false;  // the round goes on as a dense one: gossip_dense_prepare, gossip_round_compute
  return GOSSIP_OK;
}

// --- exchange dense rounds (include/gossip.h) -----------------------

namespace {
int xd_check(gossip_engine* e) {
  if (!e) return GOSSIP_EINVAL;
  if (!e->xd) return e->fail(GOSSIP_ENOTSUP, "exchange dense rounds need G > 1, W == 1 and a random mode");
  if (!e->xd_planned) return e->fail(GOSSIP_ESTATE, "gossip_sharded_plan did not plan an exchange round");
  return set_dev(e);
}
}  // namespace

int gossip_xd_classes(gossip_engine_t* e, void** send, void** image, uint64_t* bytes) {
  if (!send || !image || !bytes) return GOSSIP_EINVAL;
  if (int rc = xd_check(e)) return rc;
  *send = *image = nullptr;
  *bytes = 0;
  if (!e->xd_filt) return GOSSIP_OK;  // no filter this round: nothing to gather
  const uint64_t nwl = (e->Nl + 63) / 64;
  if (!e->xd_cls) {
    HIP_OK(e, hipMalloc((void**)&e->xd_cls, (size_t)e->G * 2 * nwl * 8));
    HIP_OK(e, hipMemsetAsync(e->xd_cls, 0, (size_t)e->G * 2 * nwl * 8, e->stream));
    HIP_OK(e, hipMalloc((void**)&e->xd_keep, e->nown + 1));
  }
  if (int rc = sx_prepare(e)) return rc;  // exact occupancy bitmaps of S_t
  uint64_t* own = e->xd_cls + (size_t)e->rank * 2 * nwl;
  const uint64_t nwo = (e->nown + 63) / 64;  // (a short last shard: its tail words stay zero)
  HIP_OK(e, hipMemcpyAsync(own, e->lf.nzb, nwo * 8, hipMemcpyDeviceToDevice, e->stream));
  HIP_OK(e, hipMemcpyAsync(own + nwl, e->lf.fullb, nwo * 8, hipMemcpyDeviceToDevice, e->stream));
  if (!e->driven && !e->ordered) HIP_OK(e, hipStreamSynchronize(e->stream));
  e->xd_cls_ok = true;
  *send = own;
  *image = e->xd_cls;
  *bytes = 2 * nwl * 8;
  return GOSSIP_OK;
}

namespace {
int xd_requests_enqueue(gossip_engine* e) {
  // a filtering round reads the gathered bitmaps: without gossip_xd_classes it runs unfiltered
  // (the filter only drops edges that move nothing, so either way the round is the same)
  const XdFilter xf{e->xd_cls, (uint32_t)((e->Nl + 63) / 64), e->xd_cls_ok ? e->xd_filt : 0u, e->xd_keep};
  if (!e->xd_smem) {
    const size_t bytes = xd_send_bytes(e->xg);
    if (hipMalloc(&e->xd_smem, bytes) != hipSuccess) {
      e->xd_smem = nullptr;
      return e->fail(GOSSIP_ENOMEM, "hipMalloc of %zu bytes (exchange send buffers) failed", bytes);
    }
    xd_carve_send(e->xg, e->xd_smem, &e->xb);
  }
  HIP_OK(e, hipMemsetAsync(e->partial_d, 0, part_len(e) * 8, e->stream));
  if (int rc = timer_begin(e, 0)) return rc;
  HIP_OK(e, launch_xd_requests(e->xg, e->xb, e->S, e->R, e->t, e->key0, e->key1, e->mode, e->fa, xf, e->stream));
  return timer_end(e, 0);
}
}  // namespace

int gossip_xd_requests(gossip_engine_t* e, void** ids, void** vals, uint64_t* send_counts) {
  if (!ids || !vals || !send_counts) return GOSSIP_EINVAL;
  if (int rc = xd_check(e)) return rc;
  if (int rc = xd_requests_enqueue(e)) return rc;
  HIP_OK(e, hipMemcpyAsync(e->xd_cnt_h, e->xb.ocnt, e->G * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  if (int rc = timer_collect(e, false)) return rc;
  for (uint32_t q = 0; q < e->G; ++q) send_counts[q] = e->xd_cnt_h[q];
  *ids = e->xb.sid;
  *vals = e->xb.sval;
  return GOSSIP_OK;
}

int gossip_xd_requests_dev(gossip_engine_t* e, void** ids, void** vals, const uint64_t** send_counts) {
  if (!ids || !vals || !send_counts) return GOSSIP_EINVAL;
  if (int rc = xd_check(e)) return rc;
  if (int rc = pub_alloc(e)) return rc;
  if (int rc = xd_requests_enqueue(e)) return rc;
  HIP_OK(e, launch_publish(nullptr, e->xb.ocnt, pub_counts(e), e->G, -1, 0, e->stream));
  if (int rc = pub_ready(e, true, false)) return rc;
  *send_counts = pub_counts(e);
  *ids = e->xb.sid;
  *vals = e->xb.sval;
  return GOSSIP_OK;
}

int gossip_xd_request_recv(gossip_engine_t* e, uint64_t items, void** ids, void** vals) {
  if (!ids || !vals) return GOSSIP_EINVAL;
  if (int rc = xd_check(e)) return rc;
  if (items >= (1ull << 31)) return e->fail(GOSSIP_EINVAL, "%llu items exceed one exchange round", (unsigned long long)items);
  if (!e->xd_rmem || items > e->xd_rcap) {
    HIP_OK(e, hipStreamSynchronize(e->stream));
    if (e->xd_rmem) HIP_OK(e, hipFree(e->xd_rmem));
    e->xd_rmem = nullptr;
    e->xd_rcap = 0;
    const uint64_t want = std::min<uint64_t>(std::max<uint64_t>(items + items / 4, kXdBinRegion), (1ull << 31) - 1);
    const size_t bytes = xd_recv_bytes(e->xg, want);
    if (hipMalloc(&e->xd_rmem, bytes) != hipSuccess) {
      e->xd_rmem = nullptr;
      return e->fail(GOSSIP_ENOMEM, "hipMalloc of %zu bytes (exchange receive buffers) failed", bytes);
    }
    xd_carve_recv(e->xg, want, e->xd_rmem, &e->xb);
    e->xd_rcap = want;
  }
  e->xd_nin = items;
  *ids = e->xb.rid;
  *vals = e->xb.rval;
  return GOSSIP_OK;
}

int gossip_xd_serve(gossip_engine_t* e, void** replies) {
  if (!replies) return GOSSIP_EINVAL;
  if (int rc = xd_check(e)) return rc;
  if (!e->xd_rmem) return e->fail(GOSSIP_ESTATE, "gossip_xd_request_recv first");
  if (int rc = timer_begin(e, 0)) return rc;
  HIP_OK(e, launch_xd_serve(e->xg, e->xb, e->S, e->xd_nin, e->R, e->stream));
  if (int rc = timer_end(e, 0)) return rc;
  if (!e->driven && !e->ordered) HIP_OK(e, hipStreamSynchronize(e->stream));
  if (int rc = timer_collect(e, false)) return rc;
  *replies = e->xb.rep_out;
  return GOSSIP_OK;
}

int gossip_xd_response_recv(gossip_engine_t* e, void** replies) {
  if (!replies) return GOSSIP_EINVAL;
  if (int rc = xd_check(e)) return rc;
  if (!e->xd_smem) return e->fail(GOSSIP_ESTATE, "gossip_xd_requests first");
  *replies = e->xb.rep_in;  // room for every own item (k x nown)
  return GOSSIP_OK;
}

namespace {
int xd_finish_enqueue(gossip_engine* e) {
  if (!e->xd_smem || !e->xd_rmem) return e->fail(GOSSIP_ESTATE, "gossip_xd_finish before the exchange");
  if (int rc = timer_begin(e, 0)) return rc;
  HIP_OK(e, launch_xd_apply(e->xg, e->xb, e->S, e->Snext, e->xd_nin, e->partial_d, e->R, e->mode, e->cfg.flags,
                            e->lf.nzb, e->lf.fullb, e->stream));
  return timer_end(e, 0);
}
void xd_finished(gossip_engine* e) {
  e->sx_valid = true;  // totals of the own nodes and exact bitmaps of S_{t+1}, fused into the apply
  e->xd_planned = e->xd_cls_ok = false;
  e->last_sparse = false;
}
}  // namespace

int gossip_xd_finish(gossip_engine_t* e, uint64_t* partial) {
  if (!partial) return GOSSIP_EINVAL;
  if (int rc = xd_check(e)) return rc;
  if (int rc = xd_finish_enqueue(e)) return rc;
  if (int rc = copy_partial_out(e, partial)) return rc;
  if (int rc = timer_collect(e)) return rc;
  xd_finished(e);
  return GOSSIP_OK;
}

int gossip_xd_finish_dev(gossip_engine_t* e, const uint64_t** partial) {
  if (!partial) return GOSSIP_EINVAL;
  if (int rc = xd_check(e)) return rc;
  if (int rc = pub_alloc(e)) return rc;
  if (int rc = xd_finish_enqueue(e)) return rc;
  if (int rc = pub_partial_out(e)) return rc;
  if (int rc = pub_ready(e, true)) return rc;
  xd_finished(e);
  *partial = pub_partial(e);
  return GOSSIP_OK;
}

// --- sharded ANTIENTROPY (include/gossip.h) -------------------------

namespace {
int aex_check(gossip_engine* e) {
  if (!e) return GOSSIP_EINVAL;
  if (!e->aex) return e->fail(GOSSIP_ENOTSUP, "gossip_ae_* calls drive sharded ANTIENTROPY engines (G > 1)");
  return set_dev(e);
}
}  // namespace

uint32_t gossip_ae_item_words(const gossip_engine_t* e, uint32_t which) {
  if (!e || !e->aex) return 0;
  return which == 0 ? e->aex_rw : e->aex_pw;
}

int gossip_ae_local_target(gossip_engine_t* e, uint32_t* out) {
  if (!out) return GOSSIP_EINVAL;
  if (int rc = aex_check(e)) return rc;
  HIP_OK(e, launch_aex_local_max(e->V, e->nown, e->R, e->aex_tmp, e->stream));
  HIP_OK(e, hipMemcpyAsync(e->partial_h, e->aex_tmp, e->R * 4, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  std::memcpy(out, e->partial_h, e->R * 4);
  return GOSSIP_OK;
}

int gossip_ae_set_target(gossip_engine_t* e, const uint32_t* target) {
  if (!target) return GOSSIP_EINVAL;
  if (int rc = aex_check(e)) return rc;
  std::memcpy(e->partial_h, target, e->R * 4);
  HIP_OK(e, hipMemcpyAsync(e->target, e->partial_h, e->R * 4, hipMemcpyHostToDevice, e->stream));
  HIP_OK(e, launch_aex_stale(make_aex_args(e), e->V, e->stream));  // own stale words of S_t
  HIP_OK(e, hipStreamSynchronize(e->stream));
  e->aex_target_ok = true;
  e->aex_inc_ok = false;  // (the next round's stats: a full pass)
  return GOSSIP_OK;
}

int gossip_ae_requests(gossip_engine_t* e, void** send, uint64_t* send_counts) {
  if (!send || !send_counts) return GOSSIP_EINVAL;
  if (int rc = aex_check(e)) return rc;
  if (!e->aex_target_ok) return e->fail(GOSSIP_ESTATE, "the global max vector is stale: gossip_ae_set_target first");
  if (e->aex_churned != e->t) return e->fail(GOSSIP_ESTATE, "gossip_exchange_buffers (and its all-gather) first");
  const AexArgs a = make_aex_args(e);
  HIP_OK(e, hipMemsetAsync(e->partial_d, 0, part_len(e) * 8, e->stream));
  // S_{t+1} starts as S_t (max only grows): the rows the last round raised, or every row
  HIP_OK(e, launch_aex_seed_next(a, e->aex_dirty, e->aex_patch_ok, e->stream));
  e->aex_patch_ok = e->aex_round_done = e->aex_track = false;
  if (int rc = timer_begin(e, 0)) return rc;
  HIP_OK(e, launch_aex_requests(a, e->stream));
  HIP_OK(e, hipMemcpyAsync(e->aex_cnt_h, e->aex_cnt, (e->G + 1) * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  uint64_t nreq = 0;
  for (uint32_t q = 0; q < e->G; ++q) {
    send_counts[q] = e->aex_cnt_h[q];
    nreq += e->aex_cnt_h[q];
  }
  e->aex_nreq = nreq;
  e->aex_nloc = e->aex_cnt_h[e->G];
  *send = e->aex_req;
  return GOSSIP_OK;
}

int gossip_ae_request_recv(gossip_engine_t* e, uint64_t items, void** recv) {
  if (!recv) return GOSSIP_EINVAL;
  if (int rc = aex_check(e)) return rc;
  if (items > e->aex_in_cap || !e->aex_in) {  // grow both the inbox and the replies to it
    const uint64_t want = std::max<uint64_t>(items + items / 4, 1024);
    for (uint32_t** b : {&e->aex_in, &e->aex_resp_out})
      if (*b) {
        HIP_OK(e, hipFree(*b));
        *b = nullptr;
      }
    e->aex_in_cap = 0;
    HIP_OK(e, hipMalloc((void**)&e->aex_in, want * e->aex_rw * 4));
    HIP_OK(e, hipMalloc((void**)&e->aex_resp_out, want * e->aex_pw * 4));
    e->aex_in_cap = want;
  }
  e->aex_nin = items;
  // few items (each raises at most one own row): mark the raised rows so the next round seeds
  // S_{t+2} from them alone; many: it copies every row (atomics on the marks would cost more)
  e->aex_track = e->aex_nreq + 2 * e->aex_nloc + items <= e->nown / 16;
  *recv = e->aex_in;
  return GOSSIP_OK;
}

int gossip_ae_serve(gossip_engine_t* e, void** send) {
  if (!send) return GOSSIP_EINVAL;
  if (int rc = aex_check(e)) return rc;
  if (!e->aex_in) return e->fail(GOSSIP_ESTATE, "gossip_ae_request_recv first");
  HIP_OK(e, launch_aex_serve(make_aex_args(e), e->aex_in, e->aex_nin, e->aex_resp_out, e->stream));
  if (!e->driven && !e->ordered) HIP_OK(e, hipStreamSynchronize(e->stream));
  *send = e->aex_resp_out;
  return GOSSIP_OK;
}

int gossip_ae_response_recv(gossip_engine_t* e, void** recv) {
  if (!recv) return GOSSIP_EINVAL;
  if (int rc = aex_check(e)) return rc;
  *recv = e->aex_resp_in;  // room for every own request (nown * k items)
  return GOSSIP_OK;
}

int gossip_ae_finish(gossip_engine_t* e, uint64_t* partial) {
  if (!partial) return GOSSIP_EINVAL;
  if (int rc = aex_check(e)) return rc;
  const bool inc = e->aex_inc_ok && e->aex_track;  // a round with few items: stats over its raised rows
  HIP_OK(e, launch_aex_finish(make_aex_args(e), e->aex_resp_in, e->aex_nreq, e->aex_nloc, inc, e->stream));
  if (int rc = timer_end(e, 0)) return rc;
  HIP_OK(e, hipMemcpyAsync(e->partial_h, e->partial_d, part_len(e) * 8, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  if (int rc = timer_collect(e)) return rc;
  std::memcpy(partial, e->partial_h, part_len(e) * 8);
  partial[4 + e->R] = 0;  // (nonzero count: random modes only)
  if (inc) partial[3] += e->aex_hash_own;  // the kernel added the raised rows' hash delta
  e->aex_hash_own = partial[3];
  e->aex_inc_ok = true;
  e->last_sparse = false;
  e->aex_round_done = e->aex_track;
  e->aex_track = false;
  return GOSSIP_OK;
}

int gossip_set_faults(gossip_engine_t* e, uint32_t edge_loss, uint32_t partitions) {
  if (!e) return GOSSIP_EINVAL;
  if ((edge_loss || partitions > 1) &&
      (e->mode == GOSSIP_MODE_ANTIENTROPY || (e->mode == GOSSIP_MODE_FLOOD && !e->flood_edges)))
    return e->fail(GOSSIP_ENOTSUP, "faults: random modes, or a FLOOD engine created with faults or stall_rounds "
                                   "(its per-edge retry state)");
  e->fa = Faults{edge_loss, partitions, e->N, e->stall_d, e->cfg.stall_rounds};
  return GOSSIP_OK;
}

}  // extern "C"

namespace {
// Marks the engines as driven by the library for the duration of one sharded_step
// (RCCL: every collective on the engines' streams; copies: the transport drains them).
struct DrivenScope {
  std::vector<gossip_engine_t*> eng;
  explicit DrivenScope(const std::vector<gossip_engine_t*>& l) : eng(l) {
    for (gossip_engine_t* e : eng) e->driven = true;
  }
  ~DrivenScope() {
    for (gossip_engine_t* e : eng) e->driven = false;
  }
};
}  // namespace

extern "C" {

int gossip_comm_unique_id(uint8_t* id) {
  if (!id) return GOSSIP_EINVAL;
  std::string err;
  const int rc = rccl_unique_id(id, &err);
  if (rc) g_create_error = err;
  return rc;
}

int gossip_comm_init_rank(gossip_engine_t* e, const uint8_t* id) {
  if (!e || !id) return GOSSIP_EINVAL;
  if (e->G < 2) return e->fail(GOSSIP_EINVAL, "gossip_comm_init_rank: shard_count is 1");
  if (e->tr) return e->fail(GOSSIP_ESTATE, "gossip_comm_init_rank: the engine has its collectives");
  if (int rc = set_dev(e)) return rc;
  HIP_OK(e, hipStreamSynchronize(e->stream));
  std::string err;
  e->tr = make_rccl_transport({e}, id, &err);
  if (!e->tr) return e->fail(GOSSIP_ERCCL, "%s", err.c_str());
  return GOSSIP_OK;
}

int gossip_step(gossip_engine_t* e, uint32_t max_rounds, gossip_round_stats_t* stats, uint64_t* infected,
                uint32_t* rounds_done) {
  if (!e) return GOSSIP_EINVAL;
  if (rounds_done) *rounds_done = 0;
  if (e->G != 1) {  // sharded rounds over the engine's own collectives
    if (!e->tr) return e->fail(GOSSIP_ESTATE, "G > 1: gossip_comm_init_rank first (or run the round_* calls)");
    if (e->mode == GOSSIP_MODE_FLOOD && !e->has_topo) return e->fail(GOSSIP_ESTATE, "FLOOD needs a topology");
    std::string err;
    const DrivenScope ds({e});
    const int rc = sharded_step({e}, e->tr, max_rounds, stats, infected, rounds_done, &err);
    if (rc) e->err = err;
    return rc;
  }
  if (e->mode == GOSSIP_MODE_FLOOD && !e->has_topo) return e->fail(GOSSIP_ESTATE, "FLOOD needs a topology");
  if (int rc = set_dev(e)) return rc;
  if (e->binned) return step_planned(e, max_rounds, stats, infected, rounds_done);
  if (e->mode == GOSSIP_MODE_ANTIENTROPY && !e->aex) return step_ae(e, max_rounds, stats, infected, rounds_done);
  std::vector<uint64_t> part(part_len(e));
  uint32_t r = 0;
  while (r < max_rounds) {
    uint64_t *send = nullptr, *img = nullptr;
    if (int rc = prepare_send(e, &send, &img)) return rc;
    if (int rc = gossip_round_compute(e, part.data())) return rc;
    gossip_round_stats_t st;
    gossip_round_commit(e, part.data(), &st);
    if (stats) stats[r] = st;
    if (infected) std::memcpy(infected + (size_t)r * e->R, part.data() + 4, (size_t)e->R * 8);
    ++r;
    if (rounds_done) *rounds_done = r;
    // converged, or FLOOD quiescence: no message sent means S_{t+1} == S_t forever
    if (st.converged || (e->mode == GOSSIP_MODE_FLOOD && st.messages == 0)) break;
  }
  return GOSSIP_OK;
}

int gossip_read_bitset(gossip_engine_t* e, uint64_t node, uint64_t* out, uint32_t nwords) {
  if (!e || !out) return GOSSIP_EINVAL;
  if (e->mode == GOSSIP_MODE_ANTIENTROPY) return e->fail(GOSSIP_ESTATE, "ANTIENTROPY: use gossip_read_versions");
  if (node < e->lo || node >= e->hi) return e->fail(GOSSIP_EINVAL, "node %llu not in this shard", (unsigned long long)node);
  if (nwords < e->W) return e->fail(GOSSIP_EINVAL, "need %u words", e->W);
  if (int rc = set_dev(e)) return rc;
  HIP_OK(e, hipStreamSynchronize(e->stream));
  for (uint32_t w = 0; w < e->W; ++w)
    HIP_OK(e, hipMemcpy(out + w, e->S + (size_t)w * e->Nl + (node - e->lo), 8, hipMemcpyDeviceToHost));
  return GOSSIP_OK;
}

int gossip_read_shard(gossip_engine_t* e, uint64_t* out, uint64_t n_words) {
  if (!e || !out) return GOSSIP_EINVAL;
  if (e->mode == GOSSIP_MODE_ANTIENTROPY) return e->fail(GOSSIP_ESTATE, "ANTIENTROPY: use gossip_read_versions");
  if (n_words < (uint64_t)e->W * e->nown) return e->fail(GOSSIP_EINVAL, "output too small");
  if (int rc = set_dev(e)) return rc;
  HIP_OK(e, hipStreamSynchronize(e->stream));
  for (uint32_t w = 0; w < e->W; ++w)
    HIP_OK(e, hipMemcpy(out + (size_t)w * e->nown, e->S + (size_t)w * e->Nl, e->nown * 8, hipMemcpyDeviceToHost));
  return GOSSIP_OK;
}

int gossip_read_versions(gossip_engine_t* e, uint64_t node, uint32_t* out, uint32_t ncomp, uint32_t* alive) {
  if (!e || !out) return GOSSIP_EINVAL;
  if (e->mode != GOSSIP_MODE_ANTIENTROPY) return e->fail(GOSSIP_ESTATE, "read_versions needs ANTIENTROPY mode");
  if (node >= e->N || ncomp < e->R) return e->fail(GOSSIP_EINVAL, "bad node or component count");
  if (e->aex && (node < e->lo || node >= e->hi))
    return e->fail(GOSSIP_EINVAL, "node %llu not in this shard", (unsigned long long)node);
  if (int rc = set_dev(e)) return rc;
  HIP_OK(e, hipStreamSynchronize(e->stream));
  if (e->aex) {
    HIP_OK(e, hipMemcpy(out, e->V + (node - e->lo) * e->R, e->R * 4, hipMemcpyDeviceToHost));
    if (alive) {  // after the last completed round's churn (the own slot of the image)
      uint64_t w = 0;
      HIP_OK(e, hipMemcpy(&w, e->aex_img + 2 * (node / 64), 8, hipMemcpyDeviceToHost));
      *alive = (uint32_t)((w >> (node & 63)) & 1ull);
    }
    return GOSSIP_OK;
  }
  HIP_OK(e, hipMemcpy(out, e->V + node * e->R, e->R * 4, hipMemcpyDeviceToHost));
  if (alive) {
    uint64_t w = 0;
    HIP_OK(e, hipMemcpy(&w, e->alive + 2 * (node / 64), 8, hipMemcpyDeviceToHost));
    *alive = (uint32_t)((w >> (node & 63)) & 1ull);
  }
  return GOSSIP_OK;
}

int gossip_read_rows(gossip_engine_t* e, uint32_t* out, uint64_t n_values) {
  if (!e || !out) return GOSSIP_EINVAL;
  if (e->mode != GOSSIP_MODE_ANTIENTROPY) return e->fail(GOSSIP_ESTATE, "read_rows needs ANTIENTROPY mode");
  if (n_values < e->nown * e->R) return e->fail(GOSSIP_EINVAL, "output too small");
  if (int rc = set_dev(e)) return rc;
  HIP_OK(e, hipStreamSynchronize(e->stream));
  const uint32_t* src = e->aex ? e->V : e->V + e->lo * e->R;
  HIP_OK(e, hipMemcpy(out, src, e->nown * e->R * 4, hipMemcpyDeviceToHost));
  return GOSSIP_OK;
}

int gossip_shard_range(const gossip_engine_t* e, uint64_t* lo, uint64_t* hi) {
  if (!e) return GOSSIP_EINVAL;
  if (lo) *lo = e->lo;
  if (hi) *hi = e->hi;
  return GOSSIP_OK;
}

int gossip_state_hash(gossip_engine_t* e, uint64_t* out) {
  if (!e || !out) return GOSSIP_EINVAL;
  if (int rc = set_dev(e)) return rc;
  if (e->aex) {  // this shard's part: hash terms of the own rows (global ids); shards' parts add up
    AexArgs a = make_aex_args(e);
    a.flags |= GOSSIP_FLAG_HASH;
    a.Vn = e->V;
    a.write_stale = false;  // (the stale words are not wanted here)
    HIP_OK(e, hipMemsetAsync(e->partial_d, 0, part_len(e) * 8, e->stream));
    HIP_OK(e, launch_aex_finish(a, nullptr, 0, 0, false, e->stream));
    HIP_OK(e, hipMemcpyAsync(e->partial_h, e->partial_d, part_len(e) * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(e, hipStreamSynchronize(e->stream));
    *out = e->partial_h[3];
    return GOSSIP_OK;
  }
  if (e->mode == GOSSIP_MODE_ANTIENTROPY) {  // the stats kernel's hash of the current rows
    AeArgs a = make_ae_args(e);
    a.flags |= GOSSIP_FLAG_HASH;
    HIP_OK(e, hipMemsetAsync(e->partial_d, 0, part_len(e) * 8, e->stream));
    HIP_OK(e, launch_ae_stats(a, e->V, e->alive, false, e->stream));
    HIP_OK(e, hipMemcpyAsync(e->partial_h, e->partial_d, part_len(e) * 8, hipMemcpyDeviceToHost, e->stream));
    HIP_OK(e, hipStreamSynchronize(e->stream));
    *out = e->partial_h[3];
    return GOSSIP_OK;
  }
  HIP_OK(e, hipMemsetAsync(e->scratch_d, 0, 8, e->stream));
  HIP_OK(e, launch_hash(e->S, e->Nl, e->nown, e->W, e->N, e->lo, e->scratch_d, e->stream));
  HIP_OK(e, hipMemcpyAsync(e->partial_h, e->scratch_d, 8, hipMemcpyDeviceToHost, e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  *out = e->partial_h[0];
  return GOSSIP_OK;
}

uint32_t gossip_round_index(const gossip_engine_t* e) { return e ? e->t : 0; }

uint32_t gossip_peer(uint64_t seed, uint64_t n_nodes, uint32_t node, uint32_t round, uint32_t j) {
  const u32x4 x = philox4x32_10(u32x4{node, round, 0u, j >> 2}, (uint32_t)seed, (uint32_t)(seed >> 32));
  return peer_from_word(lane_of(x, j & 3u), n_nodes - 1, node);
}

int gossip_philox_device(gossip_engine_t* e, const uint32_t* ctr4, const uint32_t* key2, uint32_t* out4, uint32_t n) {
  if (!e || !ctr4 || !key2 || !out4) return GOSSIP_EINVAL;
  if (int rc = set_dev(e)) return rc;
  uint32_t *dc = nullptr, *dout = nullptr;
  HIP_OK(e, hipMalloc((void**)&dc, (size_t)n * 16 + 16));
  HIP_OK(e, hipMalloc((void**)&dout, (size_t)n * 16 + 16));
  HIP_OK(e, hipMemcpy(dc, ctr4, (size_t)n * 16, hipMemcpyHostToDevice));
  HIP_OK(e, launch_philox(dc, key2[0], key2[1], dout, n, e->stream));
  HIP_OK(e, hipStreamSynchronize(e->stream));
  HIP_OK(e, hipMemcpy(out4, dout, (size_t)n * 16, hipMemcpyDeviceToHost));
  HIP_OK(e, hipFree(dc));
  HIP_OK(e, hipFree(dout));
  return GOSSIP_OK;
}

int gossip_kernel_time(const gossip_engine_t* e, uint32_t which, double* total_ms, uint64_t* launches) {
  if (!e || which >= (uint32_t)kTimers) return GOSSIP_EINVAL;
  if (total_ms) *total_ms = e->time_ms[which];
  if (launches) *launches = e->launches[which];
  return GOSSIP_OK;
}

int gossip_reset_timing(gossip_engine_t* e) {
  if (!e) return GOSSIP_EINVAL;
  for (int w = 0; w < kTimers; ++w) {
    e->time_ms[w] = 0;
    e->launches[w] = 0;
  }
  for (auto& r : e->evr_round) r = -1;  // (pending per-round events are dropped with the totals)
  for (int c = 0; c < 3; ++c) {
    e->wall_ms[c] = 0;
    e->wall_n[c] = e->wall_link[c] = 0;
  }
  e->model_ms = e->model_link_ms = 0;
  e->model_rounds = 0;
  return GOSSIP_OK;
}

int gossip_plan_model(const gossip_engine_t* e, double* model_ms, double* link_ms, uint64_t* rounds, char* plan,
                      uint32_t cap) {
  if (!e || !model_ms || !link_ms || !rounds) return GOSSIP_EINVAL;
  *model_ms = e->model_ms;
  *link_ms = e->model_link_ms;
  *rounds = e->model_rounds;
  if (plan && cap) {
    const size_t n = std::min<size_t>(e->model_plan.size(), cap - 1);
    std::memcpy(plan, e->model_plan.data(), n);
    plan[n] = 0;
  }
  return GOSSIP_OK;
}

int gossip_round_wall(const gossip_engine_t* e, uint32_t cls, double* total_ms, uint64_t* rounds,
                      uint64_t* link_bytes) {
  if (!e || cls > 2) return GOSSIP_EINVAL;
  if (total_ms) *total_ms = e->wall_ms[cls];
  if (rounds) *rounds = e->wall_n[cls];
  if (link_bytes) *link_bytes = e->wall_link[cls];
  return GOSSIP_OK;
}

// --- one process for all G shards -----------------------------------

}  // extern "C"

struct gossip_group {
  std::vector<gossip_engine_t*> eng;  // by rank
  gossip::Transport* tr = nullptr;
  std::string err;
};

namespace {
thread_local std::string g_group_error;
}  // namespace

extern "C" {

void gossip_group_destroy(gossip_group_t* g) {
  if (!g) return;
  delete g->tr;  // (the communicators first: they run on the engines' streams)
  for (gossip_engine_t* e : g->eng) gossip_destroy(e);
  delete g;
}

int gossip_group_create(const gossip_config_t* cfg, uint32_t n_shards, const int32_t* devices, int32_t transport,
                        gossip_group_t** out) {
  g_group_error.clear();
  if (!cfg || !out || n_shards == 0 || transport < 0 || transport > 2) {
    g_group_error = "gossip_group_create: bad argument";
    return GOSSIP_EINVAL;
  }
  *out = nullptr;
  auto* g = new gossip_group;
  bool distinct = true;
  for (uint32_t r = 0; r < n_shards; ++r) {
    gossip_config_t c = *cfg;
    c.shard_rank = r;
    c.shard_count = n_shards;
    if (devices) c.device = devices[r];
    for (uint32_t q = 0; q < r; ++q)
      if (devices && devices[q] == devices[r]) distinct = false;
    gossip_engine_t* e = nullptr;
    if (int rc = gossip_create(&c, &e)) {
      g_group_error = std::string("shard ") + std::to_string(r) + ": " + gossip_last_error(nullptr);
      gossip_group_destroy(g);
      return rc;
    }
    g->eng.push_back(e);
  }
  if (!devices && n_shards > 1) distinct = false;
  if (n_shards > 1) {
    const bool use_rccl = transport == 1 || (transport == 0 && distinct);
    if (use_rccl && !distinct) {
      g_group_error = "gossip_group_create: RCCL needs one device per shard";
      gossip_group_destroy(g);
      return GOSSIP_EINVAL;
    }
    std::string err;
    g->tr = use_rccl ? make_rccl_transport(g->eng, nullptr, &err) : make_copy_transport(g->eng, &err);
    if (!g->tr) {
      g_group_error = err;
      gossip_group_destroy(g);
      return use_rccl ? GOSSIP_ERCCL : GOSSIP_EINVAL;
    }
  }
  *out = g;
  return GOSSIP_OK;
}

gossip_engine_t* gossip_group_engine(gossip_group_t* g, uint32_t rank) {
  return g && rank < g->eng.size() ? g->eng[rank] : nullptr;
}

int32_t gossip_group_transport(const gossip_group_t* g) { return g && g->tr ? g->tr->kind() : 0; }

int gossip_group_step(gossip_group_t* g, uint32_t max_rounds, gossip_round_stats_t* stats, uint64_t* infected,
                      uint32_t* rounds_done) {
  if (!g) return GOSSIP_EINVAL;
  if (g->eng.size() == 1) return gossip_step(g->eng[0], max_rounds, stats, infected, rounds_done);
  g->err.clear();
  const DrivenScope ds(g->eng);
  const int rc = sharded_step(g->eng, g->tr, max_rounds, stats, infected, rounds_done, &g->err);
  return rc;
}

const char* gossip_group_last_error(const gossip_group_t* g) { return g ? g->err.c_str() : g_group_error.c_str(); }

}  // extern "C"

// engine internals for the multi-GPU driver (multi.h)
namespace gossip {
hipStream_t engine_stream(gossip_engine_t* e) { return e->stream; }
int engine_device(const gossip_engine_t* e) { return e->device; }
uint32_t engine_rank(const gossip_engine_t* e) { return e->rank; }
uint32_t engine_shards(const gossip_engine_t* e) { return e->G; }
bool engine_rccl_dev(const gossip_engine_t* e) { return e->rccl_dev; }

// whole library-driven rounds (gossip_round_wall): an event on the engine's stream before the
// plan, another after the commit (whose totals the host has read: the stream is drained)
int engine_wall_begin(gossip_engine_t* e) {
  if (!e->timing) return GOSSIP_OK;
  if (!e->wall_ev[0]) {
    HIP_OK(e, hipEventCreate(&e->wall_ev[0]));
    HIP_OK(e, hipEventCreate(&e->wall_ev[1]));
  }
  HIP_OK(e, hipEventRecord(e->wall_ev[0], e->stream));
  return GOSSIP_OK;
}

int engine_wall_end(gossip_engine_t* e, uint32_t cls, uint64_t link_bytes) {
  e->wall_n[cls] += 1;
  e->wall_link[cls] += link_bytes;
  if (!e->timing || !e->wall_ev[0]) return GOSSIP_OK;
  HIP_OK(e, hipEventRecord(e->wall_ev[1], e->stream));
  HIP_OK(e, hipEventSynchronize(e->wall_ev[1]));
  float ms = 0.f;
  HIP_OK(e, hipEventElapsedTime(&ms, e->wall_ev[0], e->wall_ev[1]));
  e->wall_ms[cls] += ms;
  return GOSSIP_OK;
}
uint32_t engine_rumors(const gossip_engine_t* e) { return e->R; }
uint32_t engine_mode(const gossip_engine_t* e) { return e->mode; }
}  // namespace gossip
