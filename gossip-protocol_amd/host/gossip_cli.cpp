// gossip_cli — native host driver of libgossip_hip.so through the C ABI only
// (include/gossip.h), the way a compiled front-end (the reference is Go, bound
// with cgo: INTEGRATION.md) drives the engine.  Runs full disseminations and
// prints one JSON line per run.
//
//   gossip_cli [--nodes N] [--rumors R] [--mode push|pull|pushpull|flood-grid]
//              [--fanout K] [--seed S] [--runs M] [--hash]
//              [--shards G [--devices d0,d1,...]]   G shards in this process, every round
//                                                   driven by the library (gossip_group_*:
//                                                   RCCL over distinct devices, else copies)
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gossip.h"

static int die(gossip_engine_t* e, const char* what, int rc) {
  std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, gossip_last_error(e));
  return 1;
}

static int die_group(gossip_group_t* g, const char* what, int rc) {
  std::fprintf(stderr, "%s failed (%d): %s\n", what, rc, gossip_group_last_error(g));
  return 1;
}

int main(int argc, char** argv) {
  uint64_t nodes = 1ull << 20, seed = 0x5EED0001;
  uint32_t rumors = 1, fanout = 3, runs = 3, shards = 1;
  std::vector<int32_t> devices;
  std::string mode = "push";
  bool hash = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() { return i + 1 < argc ? argv[++i] : (char*)"0"; };
    if (a == "--nodes") nodes = std::strtoull(next(), nullptr, 0);
    else if (a == "--rumors") rumors = (uint32_t)std::strtoul(next(), nullptr, 0);
    else if (a == "--mode") mode = next();
    else if (a == "--fanout") fanout = (uint32_t)std::strtoul(next(), nullptr, 0);
    else if (a == "--seed") seed = std::strtoull(next(), nullptr, 0);
    else if (a == "--runs") runs = (uint32_t)std::strtoul(next(), nullptr, 0);
    else if (a == "--hash") hash = true;
    else if (a == "--shards") shards = (uint32_t)std::strtoul(next(), nullptr, 0);
    else if (a == "--devices") {
      for (char* p = next(); *p;) {
        devices.push_back((int32_t)std::strtol(p, &p, 0));
        if (*p == ',') ++p;
      }
    }
    else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  gossip_config_t cfg;
  std::memset(&cfg, 0, sizeof cfg);
  cfg.n_nodes = nodes;
  cfg.n_rumors = rumors;
  cfg.fanout = fanout;
  cfg.seed = seed;
  cfg.device = -1;
  cfg.shard_count = 1;
  cfg.flags = hash ? GOSSIP_FLAG_HASH : 0;
  const bool grid = mode == "flood-grid";
  cfg.mode = mode == "push" ? GOSSIP_MODE_PUSH : mode == "pull" ? GOSSIP_MODE_PULL
           : mode == "pushpull" ? GOSSIP_MODE_PUSHPULL : GOSSIP_MODE_FLOOD;
  if (shards > 1) {  // the library runs every sharded round
    if (grid) {
      std::fprintf(stderr, "--shards: random modes only\n");
      return 2;
    }
    if (!devices.empty() && devices.size() != shards) {
      std::fprintf(stderr, "--devices wants %u ordinals\n", shards);
      return 2;
    }
    gossip_group_t* g = nullptr;
    if (int rc = gossip_group_create(&cfg, shards, devices.empty() ? nullptr : devices.data(), 0, &g))
      return die_group(nullptr, "gossip_group_create", rc);
    std::vector<gossip_round_stats_t> st(4096);
    for (uint32_t run = 0; run < runs; ++run) {
      for (uint32_t r = 0; r < shards; ++r) {
        gossip_engine_t* e = gossip_group_engine(g, r);
        if (int rc = gossip_reset(e)) return die(e, "gossip_reset", rc);
        if (int rc = gossip_inject_random(e)) return die(e, "gossip_inject_random", rc);
      }
      uint32_t done = 0;
      const auto t0 = std::chrono::steady_clock::now();
      if (int rc = gossip_group_step(g, (uint32_t)st.size(), st.data(), nullptr, &done))
        return die_group(g, "gossip_group_step", rc);
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      const gossip_round_stats_t& last = st[done ? done - 1 : 0];
      std::printf("{\"run\":%u,\"mode\":\"%s\",\"nodes\":%llu,\"rumors\":%u,\"shards\":%u,\"transport\":%d,"
                  "\"rounds\":%u,\"converged\":%u,\"node_updates_per_s\":%.4e,\"seconds\":%.6f,"
                  "\"state_hash\":\"0x%016llx\"}\n",
                  run, mode.c_str(), (unsigned long long)nodes, rumors, shards, gossip_group_transport(g), done,
                  last.converged, (double)nodes * done / s, s, (unsigned long long)last.state_hash);
    }
    gossip_group_destroy(g);
    return 0;
  }
  gossip_engine_t* e = nullptr;
  if (int rc = gossip_create(&cfg, &e)) return die(nullptr, "gossip_create", rc);
  if (grid) {  // Maelstrom-style grid topology (main.go:132-149 receives it)
    const uint64_t w = (uint64_t)std::ceil(std::sqrt((double)nodes));
    std::vector<uint32_t> row{0}, col;
    for (uint64_t i = 0; i < nodes; ++i) {
      const uint64_t r = i / w, c = i % w;
      if (r > 0) col.push_back((uint32_t)(i - w));
      if (i + w < nodes) col.push_back((uint32_t)(i + w));
      if (c > 0) col.push_back((uint32_t)(i - 1));
      if (c + 1 < w && i + 1 < nodes) col.push_back((uint32_t)(i + 1));
      row.push_back((uint32_t)col.size());
    }
    if (int rc = gossip_set_topology_csr(e, row.data(), col.data(), nodes, col.size()))
      return die(e, "gossip_set_topology_csr", rc);
  }
  std::vector<gossip_round_stats_t> st(4096);
  for (uint32_t run = 0; run < runs; ++run) {
    if (int rc = gossip_reset(e)) return die(e, "gossip_reset", rc);
    if (grid || cfg.mode == GOSSIP_MODE_PUSH || rumors == 1) {
      for (uint32_t r = 0; r < rumors; ++r)
        if (int rc = gossip_inject(e, (uint64_t)r % nodes, r)) return die(e, "gossip_inject", rc);
    } else if (int rc = gossip_inject_random(e)) {
      return die(e, "gossip_inject_random", rc);
    }
    uint32_t done = 0;
    const auto t0 = std::chrono::steady_clock::now();
    if (int rc = gossip_step(e, (uint32_t)st.size(), st.data(), nullptr, &done)) return die(e, "gossip_step", rc);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const gossip_round_stats_t& last = st[done ? done - 1 : 0];
    std::printf("{\"run\":%u,\"mode\":\"%s\",\"nodes\":%llu,\"rumors\":%u,\"rounds\":%u,\"converged\":%u,"
                "\"node_updates_per_s\":%.4e,\"seconds\":%.6f,\"state_hash\":\"0x%016llx\"}\n",
                run, mode.c_str(), (unsigned long long)nodes, rumors, done, last.converged,
                (double)nodes * done / s, s, (unsigned long long)last.state_hash);
  }
  gossip_destroy(e);
  return 0;
}
