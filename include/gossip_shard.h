/*
 * gossip_shard.h — the per-kind steps of a sharded round (libgossip_hip.so, ABI v10).
 *
 * A host that drives N GPUs through gossip_step (gossip.h: the engine owns its RCCL
 * communicators) never needs this header.  It is for a host that runs the
 * collectives itself: gossip_hip.sharded drives these calls over torch.distributed
 * (RCCL, or gloo on CPU engines), and the library's own driver (csrc/multi.hip) runs the
 * same sequence.  Each round replaces, for every node at once, the per-neighbour SyncRPC
 * of (*NodeState).Gossip (main.go:81), the reference's only cross-node traffic.
 *
 * Same conventions as gossip.h: 0 or a negative gossip_status, gossip_last_error(),
 * device buffers owned by the engine and valid until the next call on it.
 */
#ifndef GOSSIP_SHARD_H_
#define GOSSIP_SHARD_H_

#include "gossip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* --- sharded rounds (G > 1, one engine per GPU) -------------
 * Per round:  gossip_exchange_buffers → all-gather(send → recv) over RCCL
 *             → gossip_round_compute → all-reduce(SUM) of the partial vector
 *             → gossip_round_commit.
 * partial layout (uint64): [0]=full_nodes [1]=alive_nodes [2]=messages
 *                          [3]=state_hash [4..4+R)=infected per rumor
 *                          [4+R]=nonzero nodes (length gossip_partial_len). */
uint64_t gossip_partial_len(const gossip_engine_t* eng);
int gossip_exchange_buffers(gossip_engine_t* eng, void** send, void** recv, uint64_t* send_bytes);
int gossip_round_compute(gossip_engine_t* eng, uint64_t* partial);
/* Optional, dense sharded rounds (after gossip_exchange_buffers, while the
 * all-gather is in flight on another stream): enqueues on the engine's stream
 * the part of the round that reads only the own slice of the image (the pull
 * pass, the push pass over the own senders, serving the own tiles);
 * gossip_round_compute then enqueues the rest.  Returns 0 and does nothing on
 * engines without that path. */
int gossip_dense_prepare(gossip_engine_t* eng);
int gossip_round_commit(gossip_engine_t* eng, const uint64_t* total, gossip_round_stats_t* stats);

/* --- sparse sharded rounds (random modes, W == 1, G > 1) ------
 * partial_len is 5 + R for these engines: [4+R] = nonzero nodes.  Each round
 * starts with gossip_sharded_plan(total = the global totals of S_t, or NULL
 * to reuse the ones the last gossip_round_commit received):
 *   kind -1: no global totals yet -> gossip_local_totals, all-reduce(SUM),
 *            plan again with the sum;
 *   kind  0: dense round -> the exchange_buffers / round_compute sequence;
 *   kind  3: exchange dense round (no state image; see the gossip_xd_* calls below);
 *   kind  4: dense round on a class-coded state all-gather (gossip_cc_* below);
 *   kind  5 / 7: replicated dense round (param "replicate"): the steps of kind 0 /
 *            kind 4, then gossip_round_compute runs the whole image's round on every rank;
 *   kind  6: replicated dense round with the image already whole: gossip_round_compute only;
 *   kind  1: sparse round:
 *     gossip_sparse_rare(&send, &count)        own rare nodes, 16-B items {node, value}
 *     all-gather of count, stride = max count
 *     gossip_sparse_rare_recv(stride, &recv)   room for G * stride items; all-gather
 *                                              stride items from every rank into it
 *     gossip_sparse_scan(counts, &send, send_counts[G])  pushes for other shards,
 *                                              grouped by owner (16-B items)
 *     all-to-all of the counts, then of the items (owner q gets send_counts[q])
 *     gossip_sparse_msg_recv(total_in, &recv)  room for the incoming items
 *     gossip_sparse_commit(total_in, partial)  -> all-reduce(SUM) -> gossip_round_commit.
 * The device buffers stay valid until the next call on the engine; the engine
 * synchronizes its stream before returning a buffer to the driver. */
int gossip_sharded_plan(gossip_engine_t* eng, const uint64_t* total, int32_t* kind);
int gossip_local_totals(gossip_engine_t* eng, uint64_t* partial);
int gossip_sparse_rare(gossip_engine_t* eng, void** send, uint64_t* count);
int gossip_sparse_rare_recv(gossip_engine_t* eng, uint64_t stride, void** recv);
int gossip_sparse_scan(gossip_engine_t* eng, const uint64_t* counts, void** send, uint64_t* send_counts);
int gossip_sparse_msg_recv(gossip_engine_t* eng, uint64_t items, void** recv);
int gossip_sparse_commit(gossip_engine_t* eng, uint64_t items, uint64_t* partial);

/* --- sharded ANTIENTROPY rounds (G > 1; DESIGN.md §5.3, "Design B") --------------
 * Rows are sharded by node id in 64-aligned blocks (Nl = ceil(ceil(N/G)/64)*64); per round
 * every shard churns its own nodes (a per-node Philox draw) and receives every shard's alive
 * bits and stale bits (row != the global max vector).  An exchange
 * (n, p_j(n,t)) between two alive nodes with a stale end whose peer lives on another
 * shard becomes one request item {p, n, V_t[n]} to p's owner, who max-merges it into p
 * and answers V_t[p], which n's owner max-merges into n.  Items are uint32 words padded
 * to 8 bytes: request = gossip_ae_item_words(eng, 0) words, response = (eng, 1).
 * Per round:
 *   gossip_sharded_plan -> kind -2: the global max vector is stale (after reset / inject):
 *        gossip_ae_local_target(out[K]) -> all-reduce(MAX) -> gossip_ae_set_target; plan again
 *   kind 2: gossip_exchange_buffers(send = the own slot: per 64 own nodes their alive bits after
 *        this round's churn and their stale bits of S_t; recv = every shard's) -> all-gather
 *        gossip_ae_requests(&send, send_counts[G])          churn + request items by owner
 *        all-to-all of the counts; gossip_ae_request_recv(total_in, &recv); all-to-all items
 *        gossip_ae_serve(&send)                             responses, in the received order
 *        gossip_ae_response_recv(&recv); all-to-all back (the counts swapped)
 *        gossip_ae_finish(partial)                          -> all-reduce(SUM) -> gossip_round_commit */
uint32_t gossip_ae_item_words(const gossip_engine_t* eng, uint32_t which);
int gossip_ae_local_target(gossip_engine_t* eng, uint32_t* out);
int gossip_ae_set_target(gossip_engine_t* eng, const uint32_t* target);
int gossip_ae_requests(gossip_engine_t* eng, void** send, uint64_t* send_counts);
int gossip_ae_request_recv(gossip_engine_t* eng, uint64_t items, void** recv);
int gossip_ae_serve(gossip_engine_t* eng, void** send);
int gossip_ae_response_recv(gossip_engine_t* eng, void** recv);
int gossip_ae_finish(gossip_engine_t* eng, uint64_t* partial);

/* --- exchange dense rounds (random modes, W == 1, G > 1) --------------
 * A dense round without the state all-gather.  Every live edge n -> p_j(n,t) of an own
 * sender becomes one item for p's owner: id = (p - owner * Nl) | GOSSIP_XD_NO_PUSH /
 * GOSSIP_XD_NO_PULL flags (uint32) and S_t[n] (uint64, 0 without a push), in two arrays.
 * The owner ORs the pushes into S_{t+1}[p] and answers each pull with S_t[p] (uint64, in
 * the received order); the sender's owner ORs the replies into S_{t+1}[n].
 * Per round, after gossip_sharded_plan -> kind 3:
 *   gossip_xd_classes(&send, &image, &bytes)          bytes > 0: this round drops the one-way
 *                                                      edges that move nothing (a pull-only edge
 *                                                      into an empty peer, a push-only edge into a
 *                                                      full one; "xd_filter_frac"; fanout <= 8): all-gather
 *                                                      bytes from every rank's send into image (the
 *                                                      own slot is send: in place).  A shard's slot,
 *                                                      nwl = ceil(Nl / 64): [nz: nwl uint64][full:
 *                                                      nwl uint64], occupancy bitmaps of S_t.
 *                                                      Skipping the call runs the round unfiltered
 *                                                      (same result, more items).
 *   gossip_xd_requests(&ids, &vals, send_counts[G])   items grouped by owner
 *   all-to-all of the counts; gossip_xd_request_recv(total_in, &ids, &vals);
 *   all-to-all of the ids (uint32) and of the values (uint64)
 *   gossip_xd_serve(&replies)                          total_in replies, received order
 *   gossip_xd_response_recv(&replies); all-to-all back (the counts swapped)
 *   gossip_xd_finish(partial)                          -> all-reduce(SUM) -> gossip_round_commit */
#define GOSSIP_XD_NO_PUSH (1u << 30)
#define GOSSIP_XD_NO_PULL (1u << 31)
int gossip_xd_classes(gossip_engine_t* eng, void** send, void** image, uint64_t* bytes);
int gossip_xd_requests(gossip_engine_t* eng, void** ids, void** vals, uint64_t* send_counts);
int gossip_xd_request_recv(gossip_engine_t* eng, uint64_t items, void** ids, void** vals);
int gossip_xd_serve(gossip_engine_t* eng, void** replies);
int gossip_xd_response_recv(gossip_engine_t* eng, void** replies);
int gossip_xd_finish(gossip_engine_t* eng, uint64_t* partial);

/* --- device-resident round values (ABI v9) ------------------------------
 * The calls above that hand the host a count vector or the partial vector read it back and
 * synchronize the engine's stream.  Their _dev forms enqueue the same work and leave the
 * values in engine memory (uint64; counts widened), so the caller's device-side collective
 * (RCCL on the engine's stream, or a torch collective on the stream gossip_set_stream bound)
 * consumes them and one host read of its result ends the exchange:
 *   gossip_round_compute_dev -> partial_len values (node count in [1], as gossip_round_compute);
 *                               random and FLOOD modes (ANTIENTROPY partials finish on the host)
 *   gossip_sparse_rare_dev   -> 1 value, the own rare count
 *   gossip_sparse_scan_dev   -> G values, the items for each owner
 *   gossip_sparse_commit_dev -> partial_len values
 *   gossip_xd_requests_dev   -> G values, the items for each owner
 *   gossip_xd_finish_dev     -> partial_len values
 * The pointer stays valid, and its values unchanged, until the next _dev call on the engine.
 * Without a driver or ordered collectives ("ordered_collectives"), and in timing mode, the
 * call synchronizes the stream before returning (the value is then final for any stream). */
int gossip_round_compute_dev(gossip_engine_t* eng, const uint64_t** partial);
int gossip_sparse_rare_dev(gossip_engine_t* eng, void** send, const uint64_t** count);
int gossip_sparse_scan_dev(gossip_engine_t* eng, const uint64_t* counts, void** send, const uint64_t** send_counts);
int gossip_sparse_commit_dev(gossip_engine_t* eng, uint64_t items, const uint64_t** partial);
int gossip_xd_requests_dev(gossip_engine_t* eng, void** ids, void** vals, const uint64_t** send_counts);
int gossip_xd_finish_dev(gossip_engine_t* eng, const uint64_t** partial);

/* --- class-coded state all-gather (random modes, W == 1, G > 1) --------
 * A dense round on the state image whose all-gather sends, per shard, its two occupancy
 * bitmaps of S_t (bit i of word w: node lo + 64w + i nonzero / full), the number of mixed
 * nodes (nonzero, not full) before each bitmap word, and the words of its mixed nodes in id
 * order; empty and full nodes are implied.  A shard's slot, nwl = ceil(Nl / 64):
 * [nz: nwl uint64][full: nwl uint64][prefix: nwl uint32, padded to 8 bytes] = bits_bytes.
 * Per round, after gossip_sharded_plan -> kind 4:
 *   gossip_cc_send(&bits, &bits_bytes, &vals, &count)  own slot, own count mixed words
 *   all-gather of count, stride = max count
 *   gossip_cc_recv(stride, &bits_image, &vals_image)   all-gather bits_bytes from every rank
 *                                                      into bits_image (the own slot is bits:
 *                                                      in place) and stride words into vals_image
 *   gossip_cc_expand(counts[G])                        the state image from the two
 *   then as kind 0 without gossip_exchange_buffers: gossip_dense_prepare (optional),
 *   gossip_round_compute -> all-reduce(SUM) -> gossip_round_commit. */
int gossip_cc_send(gossip_engine_t* eng, void** bits, uint64_t* bits_bytes, void** vals, uint64_t* count);
int gossip_cc_recv(gossip_engine_t* eng, uint64_t stride, void** bits_image, void** vals_image);
int gossip_cc_expand(gossip_engine_t* eng, const uint64_t* counts);

#ifdef __cplusplus
}
#endif
#endif /* GOSSIP_SHARD_H_ */
