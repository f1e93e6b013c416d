// gossip_cli — native host driver of libgossip_hip.so through the C ABI only
// (include/gossip.h), the way a compiled front-end (the reference is Go, bound
// with cgo: INTEGRATION.md) drives the engine.  Runs full disseminations and
// prints one JSON line per run.
//
//   gossip_cli [--nodes N] [--rumors R] [--mode push|pull|pushpull|flood-grid]
//              [--fanout K] [--seed S] [--runs M] [--hash]
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

int main(int argc, char** argv) {
  uint64_t nodes = 1ull << 20, seed = 0x5EED0001;
  uint32_t rumors = 1, fanout = 3, runs = 3;
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
