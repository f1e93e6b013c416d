// multi.h — the engine-driven multi-GPU path: the collectives of a
// sharded round behind one interface, and the round driver that uses them.
//
// Reference anchor: the only cross-node traffic of the reference is the per-neighbour
// SyncRPC of (*NodeState).Gossip (main.go:81); here each sharded round exchanges
// state images, rare-node lists, edge items or request/reply items between the shards
// (DESIGN.md §5.1-5.3), and gossip_step runs those rounds from the calling thread.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/gossip_shard.h"

namespace gossip {

// engine internals the driver needs (engine.hip)
hipStream_t engine_stream(gossip_engine_t* e);
int engine_device(const gossip_engine_t* e);
uint32_t engine_rank(const gossip_engine_t* e);
uint32_t engine_shards(const gossip_engine_t* e);
bool engine_rccl_dev(const gossip_engine_t* e);  // gossip_set_param 'rccl_dev_collectives'
int engine_wall_begin(gossip_engine_t* e);  // gossip_round_wall: a library-driven round starts
int engine_wall_end(gossip_engine_t* e, uint32_t cls, uint64_t link_bytes);  // ... and ended
uint32_t engine_rumors(const gossip_engine_t* e);
uint32_t engine_mode(const gossip_engine_t* e);

// The collectives of one sharded round, seen from the engines of this process:
// local[i] holds shard engine_rank(local[i]); a transport serves all G shards (a
// group) or one (one process per GPU).  Inputs and outputs on the host are indexed
// by local engine; per-rank vectors by global rank.  Device buffers belong to the
// engines (the engine API returns them); collectives are enqueued on the engines'
// streams and complete before the next engine call reads their output.
class Transport {
 public:
  virtual ~Transport() = default;
  virtual int32_t kind() const = 0;  // 1 RCCL, 2 device copies
  const std::string& error() const { return err_; }

  // recv[i] = G slots of `bytes`; send[i] may be engine i's own slot (in place)
  virtual int all_gather(const std::vector<void*>& recv, const std::vector<const void*>& send, size_t bytes) = 0;
  // The same all-gather, started so that work the engines enqueue before join() runs
  // beside it (RCCL: on a side stream after an event of the engine's stream; join makes
  // the engine's stream wait for it).  Transports without a side stream finish it here.
  virtual int all_gather_start(const std::vector<void*>& recv, const std::vector<const void*>& send, size_t bytes) {
    return all_gather(recv, send, bytes);
  }
  virtual int join() { return 0; }
  // all[r] = the value of rank r (every local engine contributes mine[i])
  virtual int all_gather_u64(const std::vector<uint64_t>& mine, std::vector<uint64_t>* all) = 0;
  // sendc[i][q] = items engine i sends to rank q  ->  recvc[i][q] = items engine i gets from rank q
  virtual int all_to_all_counts(const std::vector<std::vector<uint64_t>>& sendc,
                                std::vector<std::vector<uint64_t>>* recvc) = 0;
  // bytes: send[i] holds sendb[i][q] bytes for rank q in rank order; recv[i] gets recvb[i][q] from q
  virtual int all_to_all_v(const std::vector<void*>& recv, const std::vector<std::vector<uint64_t>>& recvb,
                           const std::vector<const void*>& send, const std::vector<std::vector<uint64_t>>& sendb) = 0;
  // several all-to-alls at once (one RCCL group: they share the links instead of queueing)
  struct A2A {
    std::vector<void*> recv;
    std::vector<std::vector<uint64_t>> recvb;
    std::vector<const void*> send;
    std::vector<std::vector<uint64_t>> sendb;
  };
  virtual int all_to_all_many(const std::vector<A2A>& ops) {
    for (const A2A& o : ops)
      if (int rc = all_to_all_v(o.recv, o.recvb, o.send, o.sendb)) return rc;
    return 0;
  }
  virtual int all_reduce_sum_u64(const std::vector<std::vector<uint64_t>>& mine, std::vector<uint64_t>* sum) = 0;
  virtual int all_reduce_max_u32(const std::vector<std::vector<uint32_t>>& mine, std::vector<uint32_t>* mx) = 0;

  // Device-resident values (the engines' gossip_*_dev outputs, uint64, ready on their streams):
  // the collective reads engine memory and one host read returns its result.  The defaults
  // read the values to the host and run the host forms above.
  // one[i]: engine i's value -> all[r] = rank r's
  virtual int all_gather_dev(const std::vector<const uint64_t*>& one, std::vector<uint64_t>* all);
  // cnt[i]: G values (items engine i sends to rank q) -> sendc[i] (those, on the host), recvc[i]
  virtual int all_to_all_counts_dev(const std::vector<const uint64_t*>& cnt, std::vector<std::vector<uint64_t>>* sendc,
                                    std::vector<std::vector<uint64_t>>* recvc);
  // part[i]: n values of engine i -> their sum over every rank
  virtual int all_reduce_sum_dev(const std::vector<const uint64_t*>& part, size_t n, std::vector<uint64_t>* sum);

 protected:
  int fail(int rc, const std::string& msg) {
    err_ = msg;
    return rc;
  }
  // out[i] = the n values at p[i] (engine i's memory), after its stream has produced them
  int read_dev(const std::vector<const uint64_t*>& p, size_t n, std::vector<std::vector<uint64_t>>* out);
  virtual const std::vector<gossip_engine_t*>& engines() const = 0;
  std::string err_;
};

// RCCL: one communicator per local engine (ncclCommInitRank per process, or
// ncclCommInitAll over the distinct devices of a group).
Transport* make_rccl_transport(const std::vector<gossip_engine_t*>& local, const uint8_t* unique_id,
                               std::string* err);
// Device copies between the G engines of one process (any devices).
Transport* make_copy_transport(const std::vector<gossip_engine_t*>& local, std::string* err);
int rccl_unique_id(uint8_t* out, std::string* err);

// Runs sharded rounds over the local engines until converged (FLOOD: or a round
// that sends nothing) or max_rounds; the stats are global (the same on every rank).
int sharded_step(const std::vector<gossip_engine_t*>& local, Transport* tr, uint32_t max_rounds,
                 gossip_round_stats_t* stats, uint64_t* infected, uint32_t* rounds_done, std::string* err);

}  // namespace gossip
