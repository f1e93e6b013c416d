/*
 * gossip_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the synchronous-round gossip model used as
 * the parity checker for the HIP engine.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product library
 * (libgossip_hip.so) never links or calls it.
 *
 * The reference (0xSherlokMo/gossip-protocol, Go, main.go) cannot be built or
 * run in this container (no Go toolchain, no Maelstrom JVM harness), and it
 * ships no tests or fixtures, so this oracle is pinned by:
 *   - Random123 / rocRAND Philox4x32-10 known-answer vectors,
 *   - FLOOD = BFS-ball properties of main.go's once-only forward (main.go:65-89,113),
 *   - agreement with an independent numpy restatement (oracle/numpy_ref.py),
 *     whose outputs are committed as the JSON fixtures under tests/golden.
 * Parity against the reference's own outputs is therefore "unpinned" beyond
 * those properties.
 *
 * The API mirrors include/gossip.h with an oracle_ prefix so a test drives the
 * oracle and the engine with identical calls.
 */
#ifndef GOSSIP_ORACLE_H_
#define GOSSIP_ORACLE_H_

#include <stdint.h>
#include "../include/gossip_shard.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_sim oracle_sim_t;

void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint32_t oracle_peer(uint64_t seed, uint64_t n_nodes, uint32_t node, uint32_t round, uint32_t j);
uint32_t oracle_origin(uint64_t seed, uint64_t n_nodes, uint32_t rumor);
uint64_t oracle_mix64(uint64_t z);

/* threads: 1 = scalar reference loop, >1 = OpenMP (cpu_baseline timing). */
int oracle_create(const gossip_config_t* cfg, int threads, oracle_sim_t** out);
void oracle_destroy(oracle_sim_t* s);
int oracle_set_topology_csr(oracle_sim_t* s, const uint32_t* row_ptr, const uint32_t* col,
                            uint64_t n, uint64_t n_edges);
int oracle_reset(oracle_sim_t* s);
int oracle_inject(oracle_sim_t* s, uint64_t node, uint32_t rumor);
int oracle_inject_random(oracle_sim_t* s);
int oracle_set_faults(oracle_sim_t* s, uint32_t edge_loss, uint32_t partitions);
int oracle_set_param(oracle_sim_t* s, const char* name, double value);
int oracle_step(oracle_sim_t* s, uint32_t max_rounds, gossip_round_stats_t* stats,
                uint64_t* infected, uint32_t* rounds_done);

uint64_t oracle_partial_len(const oracle_sim_t* s);
int oracle_exchange_buffers(oracle_sim_t* s, void** send, void** recv, uint64_t* send_bytes);
int oracle_round_compute(oracle_sim_t* s, uint64_t* partial);
int oracle_round_commit(oracle_sim_t* s, const uint64_t* total, gossip_round_stats_t* stats);
/* sparse sharded rounds: the protocol of include/gossip_shard.h (gossip_sharded_plan ...) */
int oracle_sharded_plan(oracle_sim_t* s, const uint64_t* total, int32_t* kind);
int oracle_local_totals(oracle_sim_t* s, uint64_t* partial);
int oracle_sparse_rare(oracle_sim_t* s, void** send, uint64_t* count);
int oracle_sparse_rare_recv(oracle_sim_t* s, uint64_t stride, void** recv);
int oracle_sparse_scan(oracle_sim_t* s, const uint64_t* counts, void** send, uint64_t* send_counts);
int oracle_sparse_msg_recv(oracle_sim_t* s, uint64_t items, void** recv);
int oracle_sparse_commit(oracle_sim_t* s, uint64_t items, uint64_t* partial);

uint32_t oracle_ae_item_words(const oracle_sim_t* s, uint32_t which);
int oracle_ae_local_target(oracle_sim_t* s, uint32_t* out);
int oracle_ae_set_target(oracle_sim_t* s, const uint32_t* target);
int oracle_ae_requests(oracle_sim_t* s, void** send, uint64_t* send_counts);
int oracle_ae_request_recv(oracle_sim_t* s, uint64_t items, void** recv);
int oracle_ae_serve(oracle_sim_t* s, void** send);
int oracle_ae_response_recv(oracle_sim_t* s, void** recv);
int oracle_ae_finish(oracle_sim_t* s, uint64_t* partial);
int oracle_read_rows(oracle_sim_t* s, uint32_t* out, uint64_t n_values);
int oracle_xd_classes(oracle_sim_t* s, void** send, void** image, uint64_t* bytes);
int oracle_xd_requests(oracle_sim_t* s, void** ids, void** vals, uint64_t* send_counts);
int oracle_xd_request_recv(oracle_sim_t* s, uint64_t items, void** ids, void** vals);
int oracle_xd_serve(oracle_sim_t* s, void** replies);
int oracle_xd_response_recv(oracle_sim_t* s, void** replies);
int oracle_xd_finish(oracle_sim_t* s, uint64_t* partial);
int oracle_cc_send(oracle_sim_t* s, void** bits, uint64_t* bits_bytes, void** vals, uint64_t* count);
int oracle_cc_recv(oracle_sim_t* s, uint64_t stride, void** bits_image, void** vals_image);
int oracle_cc_expand(oracle_sim_t* s, const uint64_t* counts);

int oracle_read_bitset(oracle_sim_t* s, uint64_t node, uint64_t* out, uint32_t nwords);
int oracle_read_shard(oracle_sim_t* s, uint64_t* out, uint64_t n_words);
int oracle_read_versions(oracle_sim_t* s, uint64_t node, uint32_t* out, uint32_t ncomp, uint32_t* alive);
int oracle_shard_range(const oracle_sim_t* s, uint64_t* lo, uint64_t* hi);
int oracle_state_hash(oracle_sim_t* s, uint64_t* out);
uint32_t oracle_round_index(const oracle_sim_t* s);

#ifdef __cplusplus
}
#endif
#endif
