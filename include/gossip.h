/*
 * gossip.h — C ABI of the MI355X gossip-round engine (libgossip_hip.so).
 *
 * This is the drop-in boundary for the dissemination hot path of
 * 0xSherlokMo/gossip-protocol.  Each entry point names the reference
 * interface it replaces (paths are relative to the reference repo root):
 *
 *   gossip_create / gossip_destroy    NodeState + MessageKeeper construction,
 *                                     main.go:22-33 (NewMessageKeeper),
 *                                     main.go:60-63,91-97 (NodeState, NewState, var State)
 *   gossip_set_topology_csr           "topology" handler, main.go:132-149
 *                                     (State.Topology = body.Topology, :142)
 *   gossip_inject / _inject_random    "broadcast" handler from a client,
 *                                     main.go:102-117 (Broadcasted :113, Append :117)
 *   gossip_step                       (*NodeState).Gossip, main.go:65-89, run as
 *                                     synchronous rounds over every node at once
 *   gossip_read_bitset                "read" handler, main.go:123-130 (Messages.All :126)
 *
 * Semantics of a round are pinned in DESIGN.md §2 ("round model").  The
 * reference has no error returns on this path (Gossip retries until acked,
 * main.go:79-87); here every call returns 0 (GOSSIP_OK) or a negative
 * gossip_status and never aborts.  gossip_last_error() has the message.
 *
 * Ownership: the engine owns every device buffer.  Host pointers passed in
 * are read during the call only and never retained (cgo pointer rule).
 * Threading: one engine is not thread-safe; serialize calls per engine
 * (the reference serializes MessageKeeper with sync.RWMutex, main.go:25).
 *
 * Plain C: fixed-width integers and pointers only, no C++ or torch types.
 */
#ifndef GOSSIP_H_
#define GOSSIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GOSSIP_ABI_VERSION 10u

/* Dissemination modes. */
enum gossip_mode {
  GOSSIP_MODE_FLOOD = 0,      /* reference-faithful: forward once to topology neighbours, main.go:65-89 */
  GOSSIP_MODE_PUSH = 1,       /* S'[p_j(n)] |= S[n]                                         */
  GOSSIP_MODE_PULL = 2,       /* S'[n] |= S[p_j(n)]                                         */
  GOSSIP_MODE_PUSHPULL = 3,   /* both, over the same Philox peers                           */
  GOSSIP_MODE_ANTIENTROPY = 4 /* version vectors, push-pull max-merge with churn */
};

enum gossip_status {
  GOSSIP_OK = 0,
  GOSSIP_EINVAL = -1, /* bad argument                                  */
  GOSSIP_EHIP = -2,   /* HIP runtime error                             */
  GOSSIP_ENOMEM = -3, /* device allocation failed                      */
  GOSSIP_ESTATE = -4, /* call out of order (e.g. FLOOD without topology) */
  GOSSIP_ENODEV = -5, /* no usable gfx950 device                        */
  GOSSIP_ENOTSUP = -6, /* mode/feature not built                        */
  GOSSIP_ERCCL = -7    /* RCCL (librccl.so.1) missing or a collective failed */
};

enum gossip_flags {
  GOSSIP_FLAG_HASH = 1u << 0,   /* compute the per-round state hash */
  GOSSIP_FLAG_TIMING = 1u << 1, /* bracket hot kernels with hipEvents (gossip_kernel_time) */
  GOSSIP_FLAG_DIRECT = 1u << 2, /* random modes: direct random-access kernels instead of the
                                   binned (LDS) pipeline — same results, for A/B checks */
  GOSSIP_FLAG_DENSE = 1u << 3,  /* random modes: every round on the dense binned pipeline, no
                                   sparse (frontier) rounds — same results, for A/B checks */
  GOSSIP_FLAG_SHARD_DIRECT = 1u << 4,  /* sharded engines: dense rounds on the direct kernels instead
                                          of the binned push / pull passes — same results, A/B */
  GOSSIP_FLAG_AE_DIRECT_SCAN = 1u << 5 /* ANTIENTROPY: sparse rounds probe the peers' bitmap words
                                          directly instead of binning by tile — same results, A/B */
};

typedef struct gossip_config {
  uint64_t n_nodes;     /* N: global node count, 2 <= N < 2^32                       */
  uint32_t n_rumors;    /* R: rumor slots, bit r of word r/64 (W = ceil(R/64) words);
                           ANTIENTROPY: K version components per node (1..64)        */
  uint32_t mode;        /* enum gossip_mode                                           */
  uint32_t fanout;      /* k: Philox peers per node per round (random modes)          */
  uint32_t flags;       /* enum gossip_flags                                          */
  uint64_t seed;        /* Philox key = {seed lo32, seed hi32}                        */
  int32_t device;       /* HIP device ordinal, -1 = current device                    */
  uint32_t shard_rank;  /* this engine owns nodes [rank*Nl, min(N,(rank+1)*Nl))        */
  uint32_t shard_count; /* G >= 1, Nl = ceil(N/G)                                     */
  uint32_t churn_fail;    /* ANTIENTROPY: P(alive -> dead) per round, as x / 2^32      */
  uint32_t churn_recover; /* ANTIENTROPY: P(dead -> alive) per round, as x / 2^32      */
  uint32_t edge_loss;   /* random modes: P(an edge's exchange is lost) per round, x / 2^32
                           (the reference's lossy SyncRPC, main.go:77-87) */
  uint32_t partitions;  /* random modes and FLOOD: 0/1 = none, P > 1 = nodes split into P
                           contiguous blocks that cannot reach each other               */
  uint32_t stall_rounds; /* 0 = off.  D > 0: the reference's deadline stall (DESIGN.md §2.9,
                           main.go:72-87: one 2 s context per neighbour, retried forever
                           once it expired).  FLOOD: a node forwards each value down its
                           topology row in order, a lost attempt holding back the later
                           neighbours; after D lost attempts on one neighbour the walk
                           never moves past it (D = 1: the reference under silent drops).
                           Random modes: a node whose exchanges were lost in D rounds in a
                           row stops initiating exchanges until reset.  <= 16.           */
} gossip_config_t;

/* Stats of one round t: they describe S_{t+1}, the state the round produced. */
typedef struct gossip_round_stats {
  uint32_t round;       /* t                                                     */
  uint32_t converged;   /* full_nodes == alive_nodes                             */
  uint64_t full_nodes;  /* nodes holding all R rumors                            */
  uint64_t alive_nodes; /* N, or the alive count after round t's churn (ANTIENTROPY) */
  uint64_t messages;    /* FLOOD: broadcast RPCs sent in round t;
                           ANTIENTROPY: exchanges between two alive nodes           */
  uint64_t state_hash;  /* GOSSIP_FLAG_HASH: Σ mix64 over nonzero words, else 0   */
} gossip_round_stats_t;

typedef struct gossip_engine gossip_engine_t;

uint32_t gossip_abi_version(void);

/* Creates an engine on cfg->device.  Fails with GOSSIP_ENODEV when no HIP
 * device is present: there is no CPU fallback in this library. */
int gossip_create(const gossip_config_t* cfg, gossip_engine_t** out);
void gossip_destroy(gossip_engine_t* eng);

/* Last error message of eng, or of the last failed gossip_create when eng is NULL. */
const char* gossip_last_error(const gossip_engine_t* eng);

/* Launch all work on this hipStream_t from now on.  NULL binds the legacy null
 * stream (torch's default stream is the null stream: its cuda_stream is 0), so a
 * caller that passes its current stream is always ordered with the work it
 * enqueues there, e.g. RCCL collectives.  The engine finishes the work on its
 * previous stream first. */
int gossip_set_stream(gossip_engine_t* eng, void* hip_stream);

/* Knobs (the library reads no environment variables).  Every value only moves time, never a
 * result bit.  Unknown names return GOSSIP_EINVAL.
 * Operational:
 *   "timing"       0 pauses, 1 resumes the timers of an engine created with GOSSIP_FLAG_TIMING
 *                  (their hipEvents between rounds cost a few µs each)
 *   "place_tries"  a binned engine with a record slab of 512 MiB or more times the serve pass of a
 *                  zero-state trial round on up to this many allocations of the slab before its first
 *                  round and keeps the fastest (default 12; 1: the first allocation).  At most two
 *                  slabs are held at once beside the kept one
 *   "ahead"        rounds enqueued ahead of the stats read back (1..7, default 2)
 *   "ae_ahead"     ANTIENTROPY, one engine: sparse rounds enqueued at once, each gated on the
 *                  device by the previous one (1..8, default 8; 1 = one round per host read)
 *   "ordered_collectives"  1: the host runs its collectives on streams ordered after the
 *                  engine's (gossip_set_stream to the collectives' launch stream), so the
 *                  per-kind calls hand out buffers without a publishing stream sync (default 0)
 *   "link_gbps"    sharded random modes: a round is sparse or dense by a per-rank cost model
 *                  of device time plus link bytes over this many GB/s per xGMI link (default
 *                  76; 0 = the fixed sparse_frac thresholds); gossip_plan_model reports it
 *   "rccl_dev_collectives"  1: the RCCL transport's collectives read the round's counts and
 *                  partials from engine memory (gossip_*_dev); default 0: one host read first
 * Path selection, for the parity tests' A/B paths (each forces a kernel path the planner would
 * otherwise choose by cost; tests/test_abi.py pins this list):
 *   "sparse_frac"  random modes: a round runs sparse when the rare class is at most this fraction
 *                  of N (default 1/16; sharded 1/4, or 1/25 before exchange rounds; < 0 never,
 *                  >= 1 always; overrides link_gbps)
 *   "alld_frac"    sparse rounds commit every group's D once k x rare >= this x N (default 1/128)
 *   "sparse_direct"  such rounds with an empty majority OR the pushes into empty peers straight
 *                  into the state (default 1; 0: into D)
 *   "mid_frac"     past 2^25 nodes sparse rounds test a peer in the mid-level summary once this
 *                  share of peers would hit the LDS summary (default 0.5)
 *   "bin_scan_frac"  sparse rounds bin their edges by peer tile and test the peers from an LDS
 *                  copy of the rare bitmap once this share of peers would hit the LDS summary
 *                  (default 0.6, past 2^25 nodes; 0: every sparse round of an engine with the dense
 *                  pipeline, at any size; > 1 never)
 *   "scan_queue"   sparse rounds resolve the edges with a possibly rare end from a per-wave queue
 *                  (default 1; 0: where they are drawn)
 *   "filter_frac"  dense rounds drop edges by the peer's class above this empty/full fraction
 *                  (default 0.3 up to 2^25 nodes; past that off: the probes miss the L2)
 *   "xd_filter_frac"  exchange dense rounds likewise (default 0.6; >= 1 never)
 *   "xd_shards"    sharded random modes: dense rounds run as exchange rounds when G >= this
 *                  (default 6; 0 = never)
 *   "replicate"    sharded random modes: a dense round runs replicated, every rank computing the
 *                  whole image in place, so the next dense round needs no collective before it
 *                  (plan kinds 5 / 6): < 0 where the link-aware model prices it
 *                  cheaper, past 2^22 nodes (default -1), 0 never, > 0 every dense round
 *   "cc_frac"      sharded random modes: dense rounds on the state image exchange it class-coded
 *                  while the mixed nodes are at most this fraction of N (default 0.75; 0 never)
 *   "ae_sparse"    ANTIENTROPY: -1 plan sparse rounds (default), 0 never, 1 whenever valid
 *   "ae_cap"       ANTIENTROPY: edge-list capacity of sparse rounds (reallocates the list)
 *   "ae_dense_bin" ANTIENTROPY: 1 dense rounds as binned in-edge gathers (default, N <= 2^26),
 *                  0 pull pass + atomicMax push pass + stats pass
 *   "ae_dense_cap" ANTIENTROPY: in-edges per LDS pass of a binned dense round (0 = 18432)
 *   "ae_dense_filter"  ANTIENTROPY: 1 binned dense rounds skip the exchanges that cannot move a
 *                  row once fewer than 90 % of the nodes are stale (default), 0 gather them all */
int gossip_set_param(gossip_engine_t* eng, const char* name, double value);

/* FLOOD peer source: directed adjacency Topology[u] = col[row_ptr[u]..row_ptr[u+1]),
 * global node ids, n == N.  Copied; never retained.  Plain FLOOD reads each row as a set;
 * an engine created with faults or stall_rounds keeps each row as listed (order and
 * repeats: the forwarding walk of main.go:72-87) and ends every walk (a
 * known divergence: the reference's in-flight goroutine keeps the row it read at main.go:72). */
int gossip_set_topology_csr(gossip_engine_t* eng, const uint32_t* row_ptr, const uint32_t* col,
                            uint64_t n, uint64_t n_edges);

/* Clears every rumor bit and sets t = 0. */
int gossip_reset(gossip_engine_t* eng);

/* Client broadcast of rumor slot `rumor` to `node` (no-op when the node is
 * outside this shard or already holds it — the dedupe of main.go:113).
 * ANTIENTROPY: a local write of key `rumor` at `node` (its version + 1). */
int gossip_inject(gossip_engine_t* eng, uint64_t node, uint32_t rumor);

/* Injects every rumor r < R at origin(r) = Philox tag-2 draw.
 * ANTIENTROPY: initial versions V[n][c] = Philox tag-3 draw & 0xFFFF. */
int gossip_inject_random(gossip_engine_t* eng);

/* Fault model for the rounds that follow: same meaning as the config fields;
 * e.g. heal a partition between steps with partitions = 0.  FLOOD with faults
 * retries undelivered values every round (one shard only). */
int gossip_set_faults(gossip_engine_t* eng, uint32_t edge_loss, uint32_t partitions);

/* Runs rounds until converged (FLOOD also: a round that sends nothing) or max_rounds
 * rounds have run.  stats: max_rounds entries or NULL; infected: max_rounds * R
 * counters (row t = per-rumor infected counts after round t) or NULL.
 * G > 1: the engine needs its collectives first (gossip_comm_init_rank below); every
 * rank calls gossip_step with the same max_rounds and gets the same global stats. */
int gossip_step(gossip_engine_t* eng, uint32_t max_rounds, gossip_round_stats_t* stats,
                uint64_t* infected, uint32_t* rounds_done);

/* --- multi-GPU driven by the engine (G > 1) -----------------------
 * The engine runs every sharded round itself — plan, collectives, kernels — so a host
 * (the cgo binding, gossipgpu) drives N GPUs through gossip_step alone.  Collectives are
 * RCCL (librccl.so.1, loaded at first use) on the engine's stream.
 *   One process (or thread) per GPU: rank 0 calls gossip_comm_unique_id and hands the
 *   bytes to every rank by its own means; each rank creates its engine (shard_rank =
 *   rank, shard_count = G, its own device) and calls gossip_comm_init_rank, then
 *   gossip_step.  (Replaces the per-neighbour SyncRPC of main.go:81 as the only
 *   cross-node traffic.)
 *   One process for all G shards: gossip_group_create makes the G engines; transport 1
 *   = RCCL (ncclCommInitAll; the devices must be distinct), 2 = device copies (any
 *   devices, also G shards on one GPU: the same protocol without RCCL), 0 = RCCL when
 *   the devices are distinct, else copies.  gossip_group_step runs the rounds.
 * The per-kind protocol calls (a host that runs its own collectives: gossip_hip.sharded over
 * torch.distributed) are declared in gossip_shard.h. */
#define GOSSIP_UNIQUE_ID_BYTES 128
int gossip_comm_unique_id(uint8_t* id);  /* GOSSIP_UNIQUE_ID_BYTES bytes out */
int gossip_comm_init_rank(gossip_engine_t* eng, const uint8_t* id);

typedef struct gossip_group gossip_group_t;
/* devices: n_shards ordinals, or NULL = cfg->device for every shard.  cfg->shard_rank and
 * cfg->shard_count are set per engine. */
int gossip_group_create(const gossip_config_t* cfg, uint32_t n_shards, const int32_t* devices, int32_t transport,
                        gossip_group_t** out);
void gossip_group_destroy(gossip_group_t* grp);
/* Engine of shard `rank` (owned by the group: inject, read, set_param ... on it). */
gossip_engine_t* gossip_group_engine(gossip_group_t* grp, uint32_t rank);
/* 1 = RCCL, 2 = device copies. */
int32_t gossip_group_transport(const gossip_group_t* grp);
int gossip_group_step(gossip_group_t* grp, uint32_t max_rounds, gossip_round_stats_t* stats, uint64_t* infected,
                      uint32_t* rounds_done);
/* Last error of the group (or of the last failed gossip_group_create when grp is NULL). */
const char* gossip_group_last_error(const gossip_group_t* grp);

/* Readout ("read" handler, main.go:123-130).  Bitset of one node (nwords >= W),
 * or the whole owned shard in logical order out[w * Nl_owned + i]. */
int gossip_read_bitset(gossip_engine_t* eng, uint64_t node, uint64_t* out, uint32_t nwords);
int gossip_read_shard(gossip_engine_t* eng, uint64_t* out, uint64_t n_words);
/* ANTIENTROPY readout: the K versions of one node (owned by this shard), and its alive flag. */
int gossip_read_versions(gossip_engine_t* eng, uint64_t node, uint32_t* out, uint32_t ncomp, uint32_t* alive);
/* ANTIENTROPY readout of every owned row: out[i * K + c] for owned node lo + i. */
int gossip_read_rows(gossip_engine_t* eng, uint32_t* out, uint64_t n_values);
/* Owned node range [lo, hi). */
int gossip_shard_range(const gossip_engine_t* eng, uint64_t* lo, uint64_t* hi);

/* Hash of the current state (same definition as the per-round hash). */
int gossip_state_hash(gossip_engine_t* eng, uint64_t* out);

/* Current round index t (rounds executed since reset). */
uint32_t gossip_round_index(const gossip_engine_t* eng);

/* Philox peer draw p_j(n, t) exactly as the kernels compute it (parity probe). */
uint32_t gossip_peer(uint64_t seed, uint64_t n_nodes, uint32_t node, uint32_t round, uint32_t j);

/* Device-side Philox4x32-10 of n counters (known-answer tests): ctr4/out4 hold
 * 4*n words, key2 = 2 words. Runs on the engine's device. */
int gossip_philox_device(gossip_engine_t* eng, const uint32_t* ctr4, const uint32_t* key2,
                         uint32_t* out4, uint32_t n);

/* GOSSIP_FLAG_TIMING: accumulated device time (ms) and count of `which`:
 * 0 = the whole S_t -> S_{t+1} transform of a round (all its kernels; binned engines: the
 *     whole gossip_step, gaps between rounds included, launches = rounds),
 * 1 = the separate stats kernel (direct path only; fused in the binned path),
 * 2 = ANTIENTROPY sparse rounds' kernels (their stats pass counts under 1; dense rounds under 0),
 * 3 = dense rounds of a binned engine: emit + transpose + serve + apply of each round,
 * 4 = sparse (frontier) rounds of a binned engine: summary + scan + commit of each round,
 * 5 = placement trial rounds of a binned engine's record slab (param place_tries; before its
 *     first round). */
int gossip_kernel_time(const gossip_engine_t* eng, uint32_t which, double* total_ms, uint64_t* launches);
int gossip_reset_timing(gossip_engine_t* eng);
/* G > 1 rounds driven by the library (gossip_step / gossip_group_step): per class of round,
 * cls 0 = dense (plan kinds 0, 3, 4), 1 = sparse (kind 1), 2 = ANTIENTROPY (kind 2), the
 * rounds run, the bytes this shard put on its links (all-gathers: (G-1) x its slice;
 * all-to-alls: what it sent to other shards; all-reduces: 2 (G-1) / G x the vector) and, with
 * GOSSIP_FLAG_TIMING, the whole rounds' time from hipEvents on the engine's stream, collectives
 * and host round trips included (gossip_kernel_time 0 is the device work alone).  Cleared by
 * gossip_reset_timing. */
int gossip_round_wall(const gossip_engine_t* eng, uint32_t cls, double* total_ms, uint64_t* rounds,
                      uint64_t* link_bytes);
/* G > 1 random modes (either driver: the library's or a host's own collectives): the planner's
 * model of the rounds it planned (ABI v10) — the modelled per-rank ms (device time
 * from the measured rates plus link bytes over link_gbps x min(G - 1, 7) xGMI links) and its link
 * part, summed since gossip_reset_timing, the rounds they cover, and the current run's plan (one
 * letter per round since round 0: S sparse, X exchange, C class-coded, D state all-gather) in
 * plan[0 .. cap), NUL-terminated.  A measured N-GPU run can be set against it round for round. */
int gossip_plan_model(const gossip_engine_t* eng, double* model_ms, double* link_ms, uint64_t* rounds, char* plan,
                      uint32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* GOSSIP_H_ */
