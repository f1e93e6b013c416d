// multi.hip — the engine-driven multi-GPU path: RCCL and
// device-copy transports, and the sharded round driver behind gossip_step (G > 1)
// and gossip_group_step.
//
// The driver is the protocol of DESIGN.md §5.1-5.3 (the same sequence
// gossip_hip/sharded.py runs over torch.distributed): every round starts with
// gossip_sharded_plan, so all ranks take the same kind of round; its collectives go
// through a Transport.  RCCL is loaded with dlopen at first use (librccl.so.1), so
// one-GPU users never need it; the copy transport runs the same protocol between
// the G engines of one process (any devices, also G shards on one GPU), which is how
// the protocol is tested on a one-GPU box.
#include "multi.h"

#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <numeric>

#include <rccl/rccl.h>

namespace gossip {

namespace {

// --- RCCL, resolved at first use ---------------------------------------------------
struct Rccl {
  bool tried = false, ok = false;
  std::string err;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl& rccl() {
  static Rccl r;
  if (r.tried) return r;
  r.tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    r.err = std::string("cannot load librccl.so.1: ") + dlerror();
    return r;
  }
  auto sym = [&](auto** fp, const char* name) {
    *reinterpret_cast<void**>(fp) = dlsym(h, name);
    if (!*fp && r.err.empty()) r.err = std::string("librccl lacks ") + name;
  };
  sym(&r.GetUniqueId, "ncclGetUniqueId");
  sym(&r.CommInitRank, "ncclCommInitRank");
  sym(&r.CommInitAll, "ncclCommInitAll");
  sym(&r.CommDestroy, "ncclCommDestroy");
  sym(&r.AllGather, "ncclAllGather");
  sym(&r.AllReduce, "ncclAllReduce");
  sym(&r.Send, "ncclSend");
  sym(&r.Recv, "ncclRecv");
  sym(&r.GroupStart, "ncclGroupStart");
  sym(&r.GroupEnd, "ncclGroupEnd");
  sym(&r.GetErrorString, "ncclGetErrorString");
  r.ok = r.err.empty();
  return r;
}

#define RCCL_OK(call)                                                                                     \
  do {                                                                                                    \
    const ncclResult_t rc_ = (call);                                                                      \
    if (rc_ != ncclSuccess) return fail(GOSSIP_ERCCL, std::string(#call) + ": " + R.GetErrorString(rc_)); \
  } while (0)
#define HIPT_OK(call)                                                                                    \
  do {                                                                                                   \
    const hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess) return fail(GOSSIP_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

}  // namespace

int Transport::read_dev(const std::vector<const uint64_t*>& p, size_t n, std::vector<std::vector<uint64_t>>* out) {
  const std::vector<gossip_engine_t*>& eng = engines();
  out->assign(eng.size(), std::vector<uint64_t>(n, 0));
  for (size_t i = 0; i < eng.size(); ++i) {
    HIPT_OK(hipSetDevice(engine_device(eng[i])));
    HIPT_OK(hipMemcpyAsync((*out)[i].data(), p[i], n * 8, hipMemcpyDeviceToHost, engine_stream(eng[i])));
    HIPT_OK(hipStreamSynchronize(engine_stream(eng[i])));
  }
  return GOSSIP_OK;
}

int Transport::all_gather_dev(const std::vector<const uint64_t*>& one, std::vector<uint64_t>* all) {
  std::vector<std::vector<uint64_t>> v;
  if (int rc = read_dev(one, 1, &v)) return rc;
  std::vector<uint64_t> mine(v.size());
  for (size_t i = 0; i < v.size(); ++i) mine[i] = v[i][0];
  return all_gather_u64(mine, all);
}

int Transport::all_to_all_counts_dev(const std::vector<const uint64_t*>& cnt, std::vector<std::vector<uint64_t>>* sendc,
                                     std::vector<std::vector<uint64_t>>* recvc) {
  if (int rc = read_dev(cnt, engine_shards(engines()[0]), sendc)) return rc;
  return all_to_all_counts(*sendc, recvc);
}

int Transport::all_reduce_sum_dev(const std::vector<const uint64_t*>& part, size_t n, std::vector<uint64_t>* sum) {
  std::vector<std::vector<uint64_t>> v;
  if (int rc = read_dev(part, n, &v)) return rc;
  return all_reduce_sum_u64(v, sum);
}

namespace {

std::vector<uint64_t> prefix(const std::vector<uint64_t>& c) {
  std::vector<uint64_t> o(c.size() + 1, 0);
  for (size_t q = 0; q < c.size(); ++q) o[q + 1] = o[q] + c[q];
  return o;
}

// One communicator per local engine, collectives on the engine's stream.
class RcclTransport final : public Transport {
 public:
  RcclTransport(const std::vector<gossip_engine_t*>& local, std::vector<ncclComm_t> comms)
      : R(rccl()), eng_(local), comm_(std::move(comms)), G_(engine_shards(local[0])) {}
  ~RcclTransport() override {
    for (size_t i = 0; i < comm_.size(); ++i) {
      (void)hipSetDevice(engine_device(eng_[i]));
      if (side_.size() > i) {
        (void)hipStreamSynchronize(side_[i]);
        (void)hipStreamDestroy(side_[i]);
        (void)hipEventDestroy(ev_in_[i]);
        (void)hipEventDestroy(ev_out_[i]);
      }
      if (scratch_.size() > i && scratch_[i]) (void)hipFree(scratch_[i]);
      (void)R.CommDestroy(comm_[i]);
    }
    if (host_) (void)hipHostFree(host_);
  }
  int32_t kind() const override { return 1; }
  const std::vector<gossip_engine_t*>& engines() const override { return eng_; }

  int all_gather_start(const std::vector<void*>& recv, const std::vector<const void*>& send, size_t bytes) override {
    if (bytes == 0) return GOSSIP_OK;
    if (side_.empty()) {  // a side stream per engine for collectives that overlap the engine's work
      for (gossip_engine_t* e : eng_) {
        HIPT_OK(hipSetDevice(engine_device(e)));
        hipStream_t s;
        hipEvent_t a, b;
        HIPT_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        HIPT_OK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
        HIPT_OK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
        side_.push_back(s);
        ev_in_.push_back(a);
        ev_out_.push_back(b);
      }
    }
    for (size_t i = 0; i < eng_.size(); ++i) {  // the side stream starts after the engine's work so far
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      HIPT_OK(hipEventRecord(ev_in_[i], engine_stream(eng_[i])));
      HIPT_OK(hipStreamWaitEvent(side_[i], ev_in_[i], 0));
    }
    RCCL_OK(R.GroupStart());
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      RCCL_OK(R.AllGather(send[i], recv[i], bytes, ncclInt8, comm_[i], side_[i]));
    }
    RCCL_OK(R.GroupEnd());
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      HIPT_OK(hipEventRecord(ev_out_[i], side_[i]));
    }
    pending_ = true;
    return GOSSIP_OK;
  }

  int join() override {
    if (!pending_) return GOSSIP_OK;
    pending_ = false;
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      HIPT_OK(hipStreamWaitEvent(engine_stream(eng_[i]), ev_out_[i], 0));
    }
    return GOSSIP_OK;
  }

  int all_gather(const std::vector<void*>& recv, const std::vector<const void*>& send, size_t bytes) override {
    if (bytes == 0) return GOSSIP_OK;
    RCCL_OK(R.GroupStart());
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      RCCL_OK(R.AllGather(send[i], recv[i], bytes, ncclInt8, comm_[i], engine_stream(eng_[i])));
    }
    RCCL_OK(R.GroupEnd());
    return GOSSIP_OK;
  }

  int all_gather_u64(const std::vector<uint64_t>& mine, std::vector<uint64_t>* all) override {
    if (int rc = scratch(G_ * 8 + 8)) return rc;
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      uint64_t* d = (uint64_t*)scratch_[i];
      HIPT_OK(hipMemcpyAsync(d + engine_rank(eng_[i]), &mine[i], 8, hipMemcpyHostToDevice, engine_stream(eng_[i])));
    }
    RCCL_OK(R.GroupStart());
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      uint64_t* d = (uint64_t*)scratch_[i];
      RCCL_OK(R.AllGather(d + engine_rank(eng_[i]), d, 1, ncclUint64, comm_[i], engine_stream(eng_[i])));
    }
    RCCL_OK(R.GroupEnd());
    all->assign(G_, 0);
    HIPT_OK(hipSetDevice(engine_device(eng_[0])));
    HIPT_OK(hipMemcpyAsync(all->data(), scratch_[0], G_ * 8, hipMemcpyDeviceToHost, engine_stream(eng_[0])));
    return sync_all();
  }

  int all_to_all_counts(const std::vector<std::vector<uint64_t>>& sendc,
                        std::vector<std::vector<uint64_t>>* recvc) override {
    if (int rc = scratch(2 * G_ * 8)) return rc;
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      HIPT_OK(hipMemcpyAsync(scratch_[i], sendc[i].data(), G_ * 8, hipMemcpyHostToDevice, engine_stream(eng_[i])));
    }
    std::vector<std::vector<uint64_t>> one(eng_.size(), std::vector<uint64_t>(G_, 8));
    std::vector<void*> rv(eng_.size());
    std::vector<const void*> sv(eng_.size());
    for (size_t i = 0; i < eng_.size(); ++i) {
      sv[i] = scratch_[i];
      rv[i] = (char*)scratch_[i] + G_ * 8;
    }
    if (int rc = all_to_all_v(rv, one, sv, one)) return rc;
    recvc->assign(eng_.size(), std::vector<uint64_t>(G_, 0));
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      HIPT_OK(hipMemcpyAsync((*recvc)[i].data(), rv[i], G_ * 8, hipMemcpyDeviceToHost, engine_stream(eng_[i])));
    }
    return sync_all();
  }

  int all_to_all_v(const std::vector<void*>& recv, const std::vector<std::vector<uint64_t>>& recvb,
                   const std::vector<const void*>& send, const std::vector<std::vector<uint64_t>>& sendb) override {
    return all_to_all_many({A2A{recv, recvb, send, sendb}});
  }

  int all_to_all_many(const std::vector<A2A>& ops) override {
    // every rank joins, also one with nothing to send or receive
    RCCL_OK(R.GroupStart());
    for (const A2A& o : ops)
      for (size_t i = 0; i < eng_.size(); ++i) {
        HIPT_OK(hipSetDevice(engine_device(eng_[i])));
        const std::vector<uint64_t> so = prefix(o.sendb[i]), ro = prefix(o.recvb[i]);
        for (uint32_t q = 0; q < G_; ++q) {
          if (o.sendb[i][q])
            RCCL_OK(R.Send((const char*)o.send[i] + so[q], o.sendb[i][q], ncclInt8, (int)q, comm_[i],
                           engine_stream(eng_[i])));
          if (o.recvb[i][q])
            RCCL_OK(R.Recv((char*)o.recv[i] + ro[q], o.recvb[i][q], ncclInt8, (int)q, comm_[i],
                           engine_stream(eng_[i])));
        }
      }
    RCCL_OK(R.GroupEnd());
    return GOSSIP_OK;
  }

  int all_reduce_sum_u64(const std::vector<std::vector<uint64_t>>& mine, std::vector<uint64_t>* sum) override {
    const size_t n = mine[0].size();
    if (int rc = scratch(n * 8)) return rc;
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      HIPT_OK(hipMemcpyAsync(scratch_[i], mine[i].data(), n * 8, hipMemcpyHostToDevice, engine_stream(eng_[i])));
    }
    RCCL_OK(R.GroupStart());
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      RCCL_OK(R.AllReduce(scratch_[i], scratch_[i], n, ncclUint64, ncclSum, comm_[i], engine_stream(eng_[i])));
    }
    RCCL_OK(R.GroupEnd());
    sum->assign(n, 0);
    HIPT_OK(hipSetDevice(engine_device(eng_[0])));
    HIPT_OK(hipMemcpyAsync(sum->data(), scratch_[0], n * 8, hipMemcpyDeviceToHost, engine_stream(eng_[0])));
    return sync_all();
  }

  int all_reduce_max_u32(const std::vector<std::vector<uint32_t>>& mine, std::vector<uint32_t>* mx) override {
    const size_t n = mine[0].size();
    if (int rc = scratch(n * 4)) return rc;
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      HIPT_OK(hipMemcpyAsync(scratch_[i], mine[i].data(), n * 4, hipMemcpyHostToDevice, engine_stream(eng_[i])));
    }
    RCCL_OK(R.GroupStart());
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      RCCL_OK(R.AllReduce(scratch_[i], scratch_[i], n, ncclUint32, ncclMax, comm_[i], engine_stream(eng_[i])));
    }
    RCCL_OK(R.GroupEnd());
    mx->assign(n, 0);
    HIPT_OK(hipSetDevice(engine_device(eng_[0])));
    HIPT_OK(hipMemcpyAsync(mx->data(), scratch_[0], n * 4, hipMemcpyDeviceToHost, engine_stream(eng_[0])));
    return sync_all();
  }

  // the device-value forms: RCCL reads engine memory, one pinned host read per local engine.
  // Unverified on distinct GPUs, so they are opt-in (gossip_set_param "rccl_dev_collectives" on
  // the first local engine); by default the base forms run (read_dev, then the host collectives).
  bool dev_on() const { return engine_rccl_dev(eng_[0]); }
  int all_gather_dev(const std::vector<const uint64_t*>& one, std::vector<uint64_t>* all) override {
    if (!dev_on()) return Transport::all_gather_dev(one, all);
    if (int rc = scratch(G_ * 8)) return rc;
    if (int rc = pinned(G_ * 8)) return rc;
    RCCL_OK(R.GroupStart());
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      RCCL_OK(R.AllGather(one[i], scratch_[i], 1, ncclUint64, comm_[i], engine_stream(eng_[i])));
    }
    RCCL_OK(R.GroupEnd());
    HIPT_OK(hipSetDevice(engine_device(eng_[0])));
    HIPT_OK(hipMemcpyAsync(host_, scratch_[0], G_ * 8, hipMemcpyDeviceToHost, engine_stream(eng_[0])));
    HIPT_OK(hipStreamSynchronize(engine_stream(eng_[0])));
    all->assign(host_, host_ + G_);
    return GOSSIP_OK;
  }

  int all_to_all_counts_dev(const std::vector<const uint64_t*>& cnt, std::vector<std::vector<uint64_t>>* sendc,
                            std::vector<std::vector<uint64_t>>* recvc) override {
    if (!dev_on()) return Transport::all_to_all_counts_dev(cnt, sendc, recvc);
    if (int rc = scratch(G_ * 8)) return rc;
    if (int rc = pinned(eng_.size() * 2 * G_ * 8)) return rc;
    RCCL_OK(R.GroupStart());  // one value to and from every rank, the own one included
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      for (uint32_t q = 0; q < G_; ++q) {
        RCCL_OK(R.Send(cnt[i] + q, 1, ncclUint64, (int)q, comm_[i], engine_stream(eng_[i])));
        RCCL_OK(R.Recv((uint64_t*)scratch_[i] + q, 1, ncclUint64, (int)q, comm_[i], engine_stream(eng_[i])));
      }
    }
    RCCL_OK(R.GroupEnd());
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      uint64_t* h = host_ + i * 2 * G_;
      HIPT_OK(hipMemcpyAsync(h, cnt[i], G_ * 8, hipMemcpyDeviceToHost, engine_stream(eng_[i])));
      HIPT_OK(hipMemcpyAsync(h + G_, scratch_[i], G_ * 8, hipMemcpyDeviceToHost, engine_stream(eng_[i])));
    }
    if (int rc = sync_all()) return rc;
    sendc->assign(eng_.size(), {});
    recvc->assign(eng_.size(), {});
    for (size_t i = 0; i < eng_.size(); ++i) {
      const uint64_t* h = host_ + i * 2 * G_;
      (*sendc)[i].assign(h, h + G_);
      (*recvc)[i].assign(h + G_, h + 2 * G_);
    }
    return GOSSIP_OK;
  }

  int all_reduce_sum_dev(const std::vector<const uint64_t*>& part, size_t n, std::vector<uint64_t>* sum) override {
    if (!dev_on()) return Transport::all_reduce_sum_dev(part, n, sum);
    if (int rc = scratch(n * 8)) return rc;
    if (int rc = pinned(n * 8)) return rc;
    RCCL_OK(R.GroupStart());  // out of place: the engines keep their own partials
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      RCCL_OK(R.AllReduce(part[i], scratch_[i], n, ncclUint64, ncclSum, comm_[i], engine_stream(eng_[i])));
    }
    RCCL_OK(R.GroupEnd());
    HIPT_OK(hipSetDevice(engine_device(eng_[0])));
    HIPT_OK(hipMemcpyAsync(host_, scratch_[0], n * 8, hipMemcpyDeviceToHost, engine_stream(eng_[0])));
    HIPT_OK(hipStreamSynchronize(engine_stream(eng_[0])));
    sum->assign(host_, host_ + n);
    return GOSSIP_OK;
  }

 private:
  int pinned(size_t bytes) {  // pinned host room for the device-value reads
    if (bytes <= host_bytes_) return GOSSIP_OK;
    if (host_) HIPT_OK(hipHostFree(host_));
    host_ = nullptr;
    host_bytes_ = 0;
    const size_t want = std::max<size_t>(bytes, 4096);
    HIPT_OK(hipHostMalloc((void**)&host_, want, hipHostMallocDefault));
    host_bytes_ = want;
    return GOSSIP_OK;
  }
  int scratch(size_t bytes) {  // a small device buffer per engine for the host-side values
    if (bytes <= scratch_bytes_) return GOSSIP_OK;
    scratch_.resize(eng_.size(), nullptr);
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      HIPT_OK(hipStreamSynchronize(engine_stream(eng_[i])));
      if (scratch_[i]) HIPT_OK(hipFree(scratch_[i]));
      HIPT_OK(hipMalloc(&scratch_[i], std::max<size_t>(bytes, 4096)));
    }
    scratch_bytes_ = std::max<size_t>(bytes, 4096);
    return GOSSIP_OK;
  }
  int sync_all() {
    for (gossip_engine_t* e : eng_) {
      HIPT_OK(hipSetDevice(engine_device(e)));
      HIPT_OK(hipStreamSynchronize(engine_stream(e)));
    }
    return GOSSIP_OK;
  }

  Rccl& R;
  std::vector<gossip_engine_t*> eng_;
  std::vector<ncclComm_t> comm_;
  uint32_t G_;
  std::vector<void*> scratch_;
  size_t scratch_bytes_ = 0;
  uint64_t* host_ = nullptr;
  size_t host_bytes_ = 0;
  std::vector<hipStream_t> side_;
  std::vector<hipEvent_t> ev_in_, ev_out_;
  bool pending_ = false;
};

// All G shards in this process: collectives are device copies on the receiving
// engine's stream (each source engine's stream is drained first).
class CopyTransport final : public Transport {
 public:
  explicit CopyTransport(const std::vector<gossip_engine_t*>& local) : eng_(local), G_((uint32_t)local.size()) {
    for (uint32_t i = 0; i < G_; ++i) by_rank_.push_back(nullptr);
    for (gossip_engine_t* e : local) by_rank_[engine_rank(e)] = e;
  }
  int32_t kind() const override { return 2; }
  const std::vector<gossip_engine_t*>& engines() const override { return eng_; }

  int all_gather(const std::vector<void*>& recv, const std::vector<const void*>& send, size_t bytes) override {
    if (bytes == 0) return GOSSIP_OK;
    if (int rc = drain()) return rc;
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      for (size_t q = 0; q < eng_.size(); ++q) {
        char* dst = (char*)recv[i] + (size_t)engine_rank(eng_[q]) * bytes;
        if (dst == send[q]) continue;  // the own slot of an in-place gather
        HIPT_OK(hipMemcpyAsync(dst, send[q], bytes, hipMemcpyDefault, engine_stream(eng_[i])));
      }
    }
    return drain();
  }

  int all_gather_u64(const std::vector<uint64_t>& mine, std::vector<uint64_t>* all) override {
    all->assign(G_, 0);
    for (size_t i = 0; i < eng_.size(); ++i) (*all)[engine_rank(eng_[i])] = mine[i];
    return GOSSIP_OK;
  }

  int all_to_all_counts(const std::vector<std::vector<uint64_t>>& sendc,
                        std::vector<std::vector<uint64_t>>* recvc) override {
    recvc->assign(eng_.size(), std::vector<uint64_t>(G_, 0));
    for (size_t i = 0; i < eng_.size(); ++i)
      for (size_t q = 0; q < eng_.size(); ++q) (*recvc)[i][engine_rank(eng_[q])] = sendc[q][engine_rank(eng_[i])];
    return GOSSIP_OK;
  }

  int all_to_all_v(const std::vector<void*>& recv, const std::vector<std::vector<uint64_t>>& recvb,
                   const std::vector<const void*>& send, const std::vector<std::vector<uint64_t>>& sendb) override {
    if (int rc = drain()) return rc;
    std::vector<uint32_t> local_of(G_);
    for (size_t i = 0; i < eng_.size(); ++i) local_of[engine_rank(eng_[i])] = (uint32_t)i;
    for (size_t i = 0; i < eng_.size(); ++i) {
      HIPT_OK(hipSetDevice(engine_device(eng_[i])));
      const uint32_t ri = engine_rank(eng_[i]);
      const std::vector<uint64_t> ro = prefix(recvb[i]);
      for (uint32_t q = 0; q < G_; ++q) {
        if (!recvb[i][q]) continue;
        const uint32_t lq = local_of[q];
        const std::vector<uint64_t> so = prefix(sendb[lq]);
        if (sendb[lq][ri] != recvb[i][q]) return fail(GOSSIP_EINVAL, "all-to-all: send and receive counts differ");
        HIPT_OK(hipMemcpyAsync((char*)recv[i] + ro[q], (const char*)send[lq] + so[ri], recvb[i][q], hipMemcpyDefault,
                               engine_stream(eng_[i])));
      }
    }
    return drain();
  }

  int all_reduce_sum_u64(const std::vector<std::vector<uint64_t>>& mine, std::vector<uint64_t>* sum) override {
    sum->assign(mine[0].size(), 0);
    for (const auto& m : mine)
      for (size_t j = 0; j < m.size(); ++j) (*sum)[j] += m[j];  // wraps like RCCL's uint64 sum
    return GOSSIP_OK;
  }

  int all_reduce_max_u32(const std::vector<std::vector<uint32_t>>& mine, std::vector<uint32_t>* mx) override {
    mx->assign(mine[0].size(), 0);
    for (const auto& m : mine)
      for (size_t j = 0; j < m.size(); ++j) (*mx)[j] = std::max((*mx)[j], m[j]);
    return GOSSIP_OK;
  }

 private:
  int drain() {
    for (gossip_engine_t* e : eng_) {
      HIPT_OK(hipSetDevice(engine_device(e)));
      HIPT_OK(hipStreamSynchronize(engine_stream(e)));
    }
    return GOSSIP_OK;
  }
  std::vector<gossip_engine_t*> eng_;
  uint32_t G_;
  std::vector<gossip_engine_t*> by_rank_;
};

// --- the round driver ---------------------------------------------------------------

struct Driver {
  const std::vector<gossip_engine_t*>& L;
  Transport* tr;
  std::string* err;
  uint32_t G;
  std::vector<uint64_t> lb;  // this round's bytes each local shard put on its links (gossip_round_wall)

  size_t n() const { return L.size(); }
  // link-byte model of the collectives (what leaves the shard's GPU): an all-gather sends its
  // slice to G - 1 shards, an all-to-all what is addressed to other shards, a ring all-reduce
  // 2 (G - 1) / G of the vector
  void lb_all_gather(uint64_t bytes) {
    for (auto& x : lb) x += bytes * (G - 1);
  }
  void lb_all_to_all(const std::vector<std::vector<uint64_t>>& sendb) {
    for (size_t i = 0; i < n(); ++i)
      for (uint32_t q = 0; q < G; ++q)
        if (q != engine_rank(L[i])) lb[i] += sendb[i][q];
  }
  void lb_all_reduce(uint64_t bytes) {
    for (auto& x : lb) x += 2 * (G - 1) * bytes / G;
  }

  int eng_fail(size_t i, int rc) {
    *err = std::string("shard ") + std::to_string(engine_rank(L[i])) + ": " + gossip_last_error(L[i]);
    return rc;
  }
  int tr_fail(int rc) {
    *err = std::string("collective: ") + tr->error();
    return rc;
  }
#define ENG(i, call)                  \
  do {                                \
    const int rc_ = (call);           \
    if (rc_) return eng_fail(i, rc_); \
  } while (0)
#define TR(call)                 \
  do {                           \
    const int rc_ = (call);      \
    if (rc_) return tr_fail(rc_); \
  } while (0)

  int plan(int32_t* kind) {
    std::vector<int32_t> k(n());
    for (size_t i = 0; i < n(); ++i) ENG(i, gossip_sharded_plan(L[i], nullptr, &k[i]));
    if (k[0] == -2) {  // ANTIENTROPY: the global max vector after an injection (ncclMax)
      const uint32_t K = engine_rumors(L[0]);
      std::vector<std::vector<uint32_t>> t(n(), std::vector<uint32_t>(K));
      for (size_t i = 0; i < n(); ++i) ENG(i, gossip_ae_local_target(L[i], t[i].data()));
      std::vector<uint32_t> mx;
      TR(tr->all_reduce_max_u32(t, &mx));
      for (size_t i = 0; i < n(); ++i) {
        ENG(i, gossip_ae_set_target(L[i], mx.data()));
        ENG(i, gossip_sharded_plan(L[i], nullptr, &k[i]));
      }
    }
    if (k[0] == -1) {  // no global totals yet (after reset / inject): sum the shards' own
      std::vector<std::vector<uint64_t>> tot(n(), std::vector<uint64_t>(gossip_partial_len(L[0])));
      for (size_t i = 0; i < n(); ++i) ENG(i, gossip_local_totals(L[i], tot[i].data()));
      std::vector<uint64_t> sum;
      TR(tr->all_reduce_sum_u64(tot, &sum));
      for (size_t i = 0; i < n(); ++i) ENG(i, gossip_sharded_plan(L[i], sum.data(), &k[i]));
    }
    for (size_t i = 1; i < n(); ++i)
      if (k[i] != k[0]) {
        *err = "shards planned different rounds";
        return GOSSIP_ESTATE;
      }
    *kind = k[0];
    return GOSSIP_OK;
  }

  // Rounds of the random modes hand their counts and partials over as device values
  // (gossip_*_dev): each exchange of them ends in one host read, so a dense round waits on the
  // host once, an exchange round twice, a sparse round three times.
  int dense(std::vector<const uint64_t*>* pd, bool cc) {
    std::vector<void*> recv(n());
    std::vector<const void*> send(n());
    if (cc) {  // class-coded state all-gather
      std::vector<void*> bits(n()), vals(n()), rvals(n());
      std::vector<uint64_t> nb(n()), cnt(n());
      for (size_t i = 0; i < n(); ++i) ENG(i, gossip_cc_send(L[i], &bits[i], &nb[i], &vals[i], &cnt[i]));
      std::vector<uint64_t> counts;
      TR(tr->all_gather_u64(cnt, &counts));
      lb_all_gather(8);
      const uint64_t stride = *std::max_element(counts.begin(), counts.end());
      for (size_t i = 0; i < n(); ++i) {
        ENG(i, gossip_cc_recv(L[i], stride, &recv[i], &rvals[i]));
        send[i] = bits[i];
      }
      lb_all_gather(nb[0] + stride * 8);
      // the bitmaps, then the mixed words, in flight while the own-slice part of the round runs
      TR(tr->all_gather_start(recv, send, nb[0]));
      if (stride) {  // (the same side stream: joined together below)
        std::vector<const void*> vs(vals.begin(), vals.end());
        TR(tr->all_gather_start(rvals, vs, stride * 8));
      }
      for (size_t i = 0; i < n(); ++i) ENG(i, gossip_dense_prepare(L[i]));
      TR(tr->join());
      for (size_t i = 0; i < n(); ++i) ENG(i, gossip_cc_expand(L[i], counts.data()));
    } else {
      std::vector<void*> s(n());
      std::vector<uint64_t> nb(n());
      for (size_t i = 0; i < n(); ++i) {
        ENG(i, gossip_exchange_buffers(L[i], &s[i], &recv[i], &nb[i]));
        send[i] = s[i];
      }
      // the state image in flight while the own-slice part of the round runs
      TR(tr->all_gather_start(recv, send, nb[0]));
      lb_all_gather(nb[0]);
      for (size_t i = 0; i < n(); ++i) ENG(i, gossip_dense_prepare(L[i]));
      TR(tr->join());
    }
    for (size_t i = 0; i < n(); ++i) ENG(i, gossip_round_compute_dev(L[i], &(*pd)[i]));
    return GOSSIP_OK;
  }

  int sparse(std::vector<const uint64_t*>* pd) {
    std::vector<void*> rare(n()), rrecv(n()), out(n()), in(n());
    std::vector<const uint64_t*> cnt(n());
    for (size_t i = 0; i < n(); ++i) ENG(i, gossip_sparse_rare_dev(L[i], &rare[i], &cnt[i]));
    std::vector<uint64_t> counts;
    TR(tr->all_gather_dev(cnt, &counts));
    const uint64_t stride = *std::max_element(counts.begin(), counts.end());
    for (size_t i = 0; i < n(); ++i) ENG(i, gossip_sparse_rare_recv(L[i], stride, &rrecv[i]));
    if (stride) TR(tr->all_gather(rrecv, std::vector<const void*>(rare.begin(), rare.end()), stride * 16));
    lb_all_gather(8 + stride * 16);
    std::vector<std::vector<uint64_t>> oc, ic;
    std::vector<const uint64_t*> sc(n());
    for (size_t i = 0; i < n(); ++i) ENG(i, gossip_sparse_scan_dev(L[i], counts.data(), &out[i], &sc[i]));
    TR(tr->all_to_all_counts_dev(sc, &oc, &ic));
    std::vector<std::vector<uint64_t>> ob(n()), ib(n());
    std::vector<uint64_t> nin(n());
    for (size_t i = 0; i < n(); ++i) {
      nin[i] = std::accumulate(ic[i].begin(), ic[i].end(), (uint64_t)0);
      ENG(i, gossip_sparse_msg_recv(L[i], nin[i], &in[i]));
      for (uint32_t q = 0; q < G; ++q) {
        ob[i].push_back(oc[i][q] * 16);
        ib[i].push_back(ic[i][q] * 16);
      }
    }
    TR(tr->all_to_all_v(in, ib, std::vector<const void*>(out.begin(), out.end()), ob));
    lb_all_gather(8);  // (the counts)
    lb_all_to_all(ob);
    for (size_t i = 0; i < n(); ++i) ENG(i, gossip_sparse_commit_dev(L[i], nin[i], &(*pd)[i]));
    return GOSSIP_OK;
  }

  int exchange(std::vector<const uint64_t*>* pd) {
    std::vector<void*> cls(n()), img(n()), ids(n()), vals(n()), rid(n()), rval(n()), rep(n()), back(n());
    std::vector<uint64_t> nb(n());
    for (size_t i = 0; i < n(); ++i) ENG(i, gossip_xd_classes(L[i], &cls[i], &img[i], &nb[i]));
    if (nb[0]) TR(tr->all_gather(img, std::vector<const void*>(cls.begin(), cls.end()), nb[0]));
    lb_all_gather(nb[0]);
    std::vector<std::vector<uint64_t>> oc, ic;
    std::vector<const uint64_t*> sc(n());
    for (size_t i = 0; i < n(); ++i) ENG(i, gossip_xd_requests_dev(L[i], &ids[i], &vals[i], &sc[i]));
    TR(tr->all_to_all_counts_dev(sc, &oc, &ic));
    std::vector<uint64_t> nin(n());
    std::vector<std::vector<uint64_t>> o4(n()), i4(n()), o8(n()), i8(n());
    for (size_t i = 0; i < n(); ++i) {
      nin[i] = std::accumulate(ic[i].begin(), ic[i].end(), (uint64_t)0);
      ENG(i, gossip_xd_request_recv(L[i], nin[i], &rid[i], &rval[i]));
      for (uint32_t q = 0; q < G; ++q) {
        o4[i].push_back(oc[i][q] * 4);
        i4[i].push_back(ic[i][q] * 4);
        o8[i].push_back(oc[i][q] * 8);
        i8[i].push_back(ic[i][q] * 8);
      }
    }
    // the ids and the values in one group: they share the links
    TR(tr->all_to_all_many({Transport::A2A{rid, i4, std::vector<const void*>(ids.begin(), ids.end()), o4},
                            Transport::A2A{rval, i8, std::vector<const void*>(vals.begin(), vals.end()), o8}}));
    for (size_t i = 0; i < n(); ++i) {
      ENG(i, gossip_xd_serve(L[i], &rep[i]));  // replies in the received order
      ENG(i, gossip_xd_response_recv(L[i], &back[i]));
    }
    // the replies go back: what engine i received from q returns to q
    TR(tr->all_to_all_v(back, o8, std::vector<const void*>(rep.begin(), rep.end()), i8));
    lb_all_gather(8);  // (the counts)
    lb_all_to_all(o4);
    lb_all_to_all(o8);
    lb_all_to_all(i8);  // the replies go back
    for (size_t i = 0; i < n(); ++i) ENG(i, gossip_xd_finish_dev(L[i], &(*pd)[i]));
    return GOSSIP_OK;
  }

  int antientropy(std::vector<std::vector<uint64_t>>* part) {
    const uint64_t rw = gossip_ae_item_words(L[0], 0), pw = gossip_ae_item_words(L[0], 1);
    std::vector<void*> s(n()), recv(n()), req(n()), inbox(n()), resp(n()), back(n());
    std::vector<uint64_t> nb(n());
    for (size_t i = 0; i < n(); ++i) ENG(i, gossip_exchange_buffers(L[i], &s[i], &recv[i], &nb[i]));
    TR(tr->all_gather(recv, std::vector<const void*>(s.begin(), s.end()), nb[0]));
    lb_all_gather(nb[0] + 8);
    std::vector<std::vector<uint64_t>> oc(n(), std::vector<uint64_t>(G)), ic;
    for (size_t i = 0; i < n(); ++i) ENG(i, gossip_ae_requests(L[i], &req[i], oc[i].data()));
    TR(tr->all_to_all_counts(oc, &ic));
    std::vector<uint64_t> nin(n());
    std::vector<std::vector<uint64_t>> oq(n()), iq(n()), op(n()), ip(n());
    for (size_t i = 0; i < n(); ++i) {
      nin[i] = std::accumulate(ic[i].begin(), ic[i].end(), (uint64_t)0);
      ENG(i, gossip_ae_request_recv(L[i], nin[i], &inbox[i]));
      for (uint32_t q = 0; q < G; ++q) {
        oq[i].push_back(oc[i][q] * rw * 4);
        iq[i].push_back(ic[i][q] * rw * 4);
        op[i].push_back(oc[i][q] * pw * 4);
        ip[i].push_back(ic[i][q] * pw * 4);
      }
    }
    TR(tr->all_to_all_v(inbox, iq, std::vector<const void*>(req.begin(), req.end()), oq));
    for (size_t i = 0; i < n(); ++i) {
      ENG(i, gossip_ae_serve(L[i], &resp[i]));  // replies in the received order
      ENG(i, gossip_ae_response_recv(L[i], &back[i]));
    }
    TR(tr->all_to_all_v(back, op, std::vector<const void*>(resp.begin(), resp.end()), ip));
    lb_all_to_all(oq);
    lb_all_to_all(ip);  // the responses go back
    for (size_t i = 0; i < n(); ++i) ENG(i, gossip_ae_finish(L[i], (*part)[i].data()));
    return GOSSIP_OK;
  }

  int round(gossip_round_stats_t* st, std::vector<uint64_t>* total) {
    lb.assign(n(), 0);
    for (size_t i = 0; i < n(); ++i) ENG(i, engine_wall_begin(L[i]));
    int32_t kind = 0;
    if (int rc = plan(&kind)) return rc;
    const size_t plen = gossip_partial_len(L[0]);
    std::vector<std::vector<uint64_t>> part;  // ANTIENTROPY: partials finished on the host
    std::vector<const uint64_t*> pd(n(), nullptr);  // the others: device values
    int rc;
    switch (kind) {
      case 1: rc = sparse(&pd); break;
      case 2:
        part.assign(n(), std::vector<uint64_t>(plen));
        rc = antientropy(&part);
        break;
      case 3: rc = exchange(&pd); break;
      case 4:
      case 7: rc = dense(&pd, true); break;  // (7: class-coded all-gather, then the replicated round)
      case 6:  // replicated, the image whole already: no collective before it
        for (size_t i = 0; i < n(); ++i) ENG(i, gossip_round_compute_dev(L[i], &pd[i]));
        rc = GOSSIP_OK;
        break;
      default: rc = dense(&pd, false); break;  // 0, 5 (the state all-gather, then the replicated round)
    }
    if (rc) return rc;
    if (kind == 2) TR(tr->all_reduce_sum_u64(part, total));
    else TR(tr->all_reduce_sum_dev(pd, plen, total));
    lb_all_reduce(plen * 8);
    for (size_t i = 0; i < n(); ++i) {
      gossip_round_stats_t s;
      ENG(i, gossip_round_commit(L[i], total->data(), &s));
      if (i == 0) *st = s;
    }
    const uint32_t cls = kind == 1 ? 1u : kind == 2 ? 2u : 0u;
    for (size_t i = 0; i < n(); ++i) ENG(i, engine_wall_end(L[i], cls, lb[i]));
    return GOSSIP_OK;
  }
#undef ENG
#undef TR
};

}  // namespace

int rccl_unique_id(uint8_t* out, std::string* err) {
  Rccl& R = rccl();
  if (!R.ok) {
    *err = R.err;
    return GOSSIP_ERCCL;
  }
  ncclUniqueId id;
  const ncclResult_t rc = R.GetUniqueId(&id);
  if (rc != ncclSuccess) {
    *err = std::string("ncclGetUniqueId: ") + R.GetErrorString(rc);
    return GOSSIP_ERCCL;
  }
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return GOSSIP_OK;
}

Transport* make_rccl_transport(const std::vector<gossip_engine_t*>& local, const uint8_t* unique_id,
                               std::string* err) {
  Rccl& R = rccl();
  if (!R.ok) {
    *err = R.err;
    return nullptr;
  }
  const uint32_t G = engine_shards(local[0]);
  std::vector<ncclComm_t> comms(local.size(), nullptr);
  ncclResult_t rc;
  if (unique_id) {  // one engine of a multi-process world
    ncclUniqueId id;
    std::memcpy(id.internal, unique_id, NCCL_UNIQUE_ID_BYTES);
    (void)hipSetDevice(engine_device(local[0]));
    rc = R.CommInitRank(&comms[0], (int)G, id, (int)engine_rank(local[0]));
  } else {  // every shard in this process, one per device, in rank order
    std::vector<int> devs(local.size());
    for (size_t i = 0; i < local.size(); ++i) devs[i] = engine_device(local[i]);
    rc = R.CommInitAll(comms.data(), (int)local.size(), devs.data());
  }
  if (rc != ncclSuccess) {
    *err = std::string(unique_id ? "ncclCommInitRank: " : "ncclCommInitAll: ") + R.GetErrorString(rc);
    return nullptr;
  }
  return new RcclTransport(local, std::move(comms));
}

Transport* make_copy_transport(const std::vector<gossip_engine_t*>& local, std::string* err) {
  if (local.size() != engine_shards(local[0])) {
    *err = "the copy transport needs every shard in this process";
    return nullptr;
  }
  for (size_t i = 0; i < local.size(); ++i)
    for (size_t j = 0; j < local.size(); ++j) {
      const int a = engine_device(local[i]), b = engine_device(local[j]);
      if (a == b) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can) {
        (void)hipSetDevice(a);
        (void)hipDeviceEnablePeerAccess(b, 0);  // hipErrorPeerAccessAlreadyEnabled is fine
        (void)hipGetLastError();
      }
    }
  return new CopyTransport(local);
}

int sharded_step(const std::vector<gossip_engine_t*>& local, Transport* tr, uint32_t max_rounds,
                 gossip_round_stats_t* stats, uint64_t* infected, uint32_t* rounds_done, std::string* err) {
  if (rounds_done) *rounds_done = 0;
  Driver d{local, tr, err, engine_shards(local[0])};
  const uint32_t R = engine_rumors(local[0]);
  const bool flood = engine_mode(local[0]) == GOSSIP_MODE_FLOOD;
  std::vector<uint64_t> total;
  for (uint32_t r = 0; r < max_rounds; ++r) {
    gossip_round_stats_t st;
    if (int rc = d.round(&st, &total)) return rc;
    if (stats) stats[r] = st;
    if (infected) std::memcpy(infected + (size_t)r * R, total.data() + 4, (size_t)R * 8);
    if (rounds_done) *rounds_done = r + 1;
    if (st.converged || (flood && st.messages == 0)) break;
  }
  return GOSSIP_OK;
}

}  // namespace gossip
