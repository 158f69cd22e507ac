// The reference's real build call shape on one GPU: many builder threads at
// once (up to 4 flush + 12 compaction + 12 subcompaction threads per compute
// node, include/TimberSaw/options.h:73-79; one std::thread per subcompaction,
// db/db_impl.cc:3373-3386), each TableBuilder owning one
// FullFilterBlockBuilder (table/table_builder_computeside.cc:62-64) that is
// driven RestartBlock / AddKey x n / Finish into its own RDMA-registered
// (here: page-locked) filter slot.  One dlsm_ctx per thread.
//
// Phases, each started by all threads together:
//   1. warm-up: one table per thread (contexts grow their workspaces);
//   2. timed GPU: `tables` tables per thread through the adapter;
//   3. timed CPU: the same tables through the oracle restatement (the
//      reference's cost structure: hash -> vector -> scatter), same threads.
// Checks every filter against the oracle (test infrastructure) and that no
// context allocates device memory after its warm-up table (dlsm_ctx_stats);
// prints per-Finish latency and both aggregate rates as one JSON line.
//
//   concurrent_builders [threads=16] [tables_per_thread=8] [keys=153846] [mode=ctx] [window_us=0]
//
// mode: ctx        -- one dlsm_ctx per thread, one synchronous build per table;
//       batch      -- Finish goes through the device's dlsm_batcher: the
//                     threads' concurrent calls become batched builds;
//       hash       -- one ctx per thread, AddKey hashes on the host (the
//                     reference's AddKey) and Finish sends 4 B per key;
//       batch-hash -- both;
//       ref        -- the reference's own signature and AddKey: builders
//                     constructed as FullFilterBlockBuilder(ibv_mr*, bits_per_key)
//                     (an ibv_mr-shaped region: addr + length), the thread's
//                     context from dlsm_thread_ctx, AddKey = BloomHash into
//                     hash_entries_ with the consecutive-duplicate drop
//                     (full_filter_block.cc:39-49), Finish = the hashed GPU build
//                     into the page-locked slot.
// Threads up to 28 = dLSM's 4 flush + 12 compaction + 12 subcompaction
// builder threads (include/TimberSaw/options.h:73,77-78).
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "dlsm_bloom_adapter.hpp"

extern "C" {
int64_t orc_full_build(const uint8_t*, const uint64_t*, uint32_t, uint64_t, int, uint8_t*, uint64_t);
void orc_dbbench_key(uint64_t v, int key_size, uint8_t* out);
}

using dlsm_adapter::Slice;
using Clock = std::chrono::steady_clock;

// Field layout of <infiniband/verbs.h>'s struct ibv_mr (context, pd, addr,
// length, handle, lkey, rkey): the reference-signature constructor reads only
// addr and length, so the real ibv_mr binds the same way.
struct IbvMrShaped {
  void* context;
  void* pd;
  void* addr;
  size_t length;
  uint32_t handle, lkey, rkey;
};

class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  // returns the time at which the last thread arrived
  Clock::time_point wait() {
    std::unique_lock<std::mutex> lk(m_);
    const int g = gen_;
    if (++count_ == n_) {
      count_ = 0;
      gen_++;
      at_ = Clock::now();
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen_ != g; });
    }
    return at_;
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  int n_, count_ = 0, gen_ = 0;
  Clock::time_point at_;
};

struct ThreadResult {
  int failures = 0;
  std::string what;
  std::vector<double> finish_ms;  // per timed table
  double add_ms = 0;              // AddKey loops of the timed tables
  uint64_t allocs_after_warmup = 0, allocs_end = 0;
  Clock::time_point gpu_start, gpu_end, cpu_start, cpu_end;
};

static void run_thread(int t, int threads, int tables, int n, Barrier* bar, ThreadResult* r,
                       dlsm_adapter::BuilderOptions opt, bool ref) {
  dlsm_ctx* ctx = nullptr;
  const int ok_ctx = (opt.batcher || ref) ? DLSM_OK : dlsm_ctx_create(0, &ctx);
  uint64_t spec = 0;
  dlsm_bloom_full_size(n, 10, nullptr, &spec);
  const size_t slot_len = 256 * 1024 > spec ? 256 * 1024 : spec;  // FilterChunk slot (options.h:28)
  const uint64_t S = static_cast<uint64_t>(tables + 1) * threads;
  // table q of thread t: db_bench keys v = sid + S*i, sid = q*threads + t
  std::vector<std::vector<uint8_t>> keys(tables + 1, std::vector<uint8_t>(static_cast<size_t>(n) * 20));
  std::vector<std::vector<uint8_t>> got(tables + 1);
  for (int q = 0; q <= tables; q++) {
    const uint64_t sid = static_cast<uint64_t>(q) * threads + t;
    for (int i = 0; i < n; i++) orc_dbbench_key(sid + S * static_cast<uint64_t>(i), 20, &keys[q][20 * static_cast<size_t>(i)]);
  }
  void* slot_mem = nullptr;
  if (ok_ctx != DLSM_OK || dlsm_host_alloc(slot_len, &slot_mem) != DLSM_OK) {
    r->failures++;
    r->what = "ctx_create / host_alloc";
  }
  dlsm_adapter::FilterSlot mr{slot_mem, slot_len};
  IbvMrShaped ibv{nullptr, nullptr, slot_mem, slot_len, 0, 0, 0};
  auto build = [&](int q, bool timed) {
    if (r->failures) return;
    dlsm_adapter::FullFilterBlockBuilder b = ref ? dlsm_adapter::FullFilterBlockBuilder(&ibv, 10)
                                                 : dlsm_adapter::FullFilterBlockBuilder(&mr, 10, ctx, opt);
    std::memset(slot_mem, 0, slot_len);  // Rep ctor memsets the slot (table_builder_computeside.cc:38)
    const auto t0 = Clock::now();
    b.RestartBlock(0);
    for (int i = 0; i < n; i++) b.AddKey(Slice(reinterpret_cast<const char*>(&keys[q][20 * static_cast<size_t>(i)]), 20));
    const auto t1 = Clock::now();
    b.Finish();
    const auto t2 = Clock::now();
    if (b.status() != DLSM_OK) {
      r->failures++;
      r->what = "finish status " + std::to_string(b.status());
      return;
    }
    got[q].assign(reinterpret_cast<const uint8_t*>(b.result.data()),
                  reinterpret_cast<const uint8_t*>(b.result.data()) + b.result.size());
    if (timed) {
      r->finish_ms.push_back(std::chrono::duration<double, std::milli>(t2 - t1).count());
      r->add_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
    }
  };
  bar->wait();
  build(0, false);  // warm-up
  if (ref) dlsm_thread_ctx(&ctx);  // the thread's context the builders took (owned by the library)
  if (!r->failures && ctx) dlsm_ctx_stats(ctx, &r->allocs_after_warmup, nullptr);
  r->gpu_start = bar->wait();
  for (int q = 1; q <= tables; q++) build(q, true);
  r->gpu_end = Clock::now();
  if (!r->failures && ctx) dlsm_ctx_stats(ctx, &r->allocs_end, nullptr);
  std::vector<std::vector<uint8_t>> want(tables + 1, std::vector<uint8_t>(spec));
  std::vector<int64_t> wl(tables + 1);
  r->cpu_start = bar->wait();
  for (int q = 1; q <= tables; q++)
    wl[q] = orc_full_build(keys[q].data(), nullptr, 20, n, 10, want[q].data(), want[q].size());
  r->cpu_end = Clock::now();
  wl[0] = orc_full_build(keys[0].data(), nullptr, 20, n, 10, want[0].data(), want[0].size());
  for (int q = 0; q <= tables && !r->failures; q++) {
    if (wl[q] != static_cast<int64_t>(got[q].size()) || std::memcmp(want[q].data(), got[q].data(), wl[q]) != 0) {
      r->failures++;
      r->what = "filter bytes differ from the oracle: thread " + std::to_string(t) + " table " + std::to_string(q);
    }
  }
  if (slot_mem) dlsm_host_free(slot_mem);
  if (ctx && !ref) dlsm_ctx_destroy(ctx);
}

int main(int argc, char** argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 16;
  const int tables = argc > 2 ? std::atoi(argv[2]) : 8;
  const int n = argc > 3 ? std::atoi(argv[3]) : 153846;
  const std::string mode = argc > 4 ? argv[4] : "ctx";
  dlsm_adapter::BuilderOptions opt;
  opt.hash_in_addkey = mode == "hash" || mode == "batch-hash";
  dlsm_batcher* batcher = nullptr;
  if (mode == "batch" || mode == "batch-hash") {
    const uint32_t window_us = argc > 5 ? static_cast<uint32_t>(std::atoi(argv[5])) : 0u;
    if (dlsm_batcher_create(0, 2, window_us, 64, &batcher) != DLSM_OK) {
      std::printf("FAIL batcher_create\n");
      return 1;
    }
    opt.batcher = batcher;
  } else if (mode != "ctx" && mode != "hash" && mode != "ref") {
    std::printf("FAIL unknown mode %s\n", mode.c_str());
    return 1;
  }
  std::vector<ThreadResult> res(threads);
  Barrier bar(threads);
  std::vector<std::thread> th;
  for (int t = 0; t < threads; t++) th.emplace_back(run_thread, t, threads, tables, n, &bar, &res[t], opt, mode == "ref");
  for (auto& x : th) x.join();
  uint64_t nb = 0, nj = 0, mb = 0;
  if (batcher) {
    dlsm_batcher_stats(batcher, &nb, &nj, &mb);
    dlsm_batcher_destroy(batcher);
  }
  int fails = 0;
  std::vector<double> lat;
  double add_ms = 0;
  bool no_alloc = true;
  Clock::time_point gs = res[0].gpu_start, ge = res[0].gpu_end, cs = res[0].cpu_start, ce = res[0].cpu_end;
  for (auto& r : res) {
    fails += r.failures;
    if (r.failures) std::printf("thread failure: %s\n", r.what.c_str());
    lat.insert(lat.end(), r.finish_ms.begin(), r.finish_ms.end());
    add_ms += r.add_ms;
    no_alloc = no_alloc && r.allocs_end == r.allocs_after_warmup;
    ge = std::max(ge, r.gpu_end);
    ce = std::max(ce, r.cpu_end);
  }
  // Finish calls over 2 ms, by the thread's table index (1 = its first timed table)
  std::string slow = "[";
  for (int q = 0; q < tables; q++) {
    int c = 0;
    for (auto& r : res) c += q < static_cast<int>(r.finish_ms.size()) && r.finish_ms[q] > 2.0;
    slow += (q ? ", " : "") + std::to_string(c);
  }
  slow += "]";
  const char* hs = std::getenv("DLSM_HOST_SYNC");
  std::sort(lat.begin(), lat.end());
  const auto pct = [&](double p) { return lat.empty() ? 0.0 : lat[std::min(lat.size() - 1, static_cast<size_t>(p * lat.size()))]; };
  double sum = 0;
  for (double x : lat) sum += x;
  const double keys_timed = static_cast<double>(threads) * tables * n;
  const double gpu_ms = std::chrono::duration<double, std::milli>(ge - gs).count();
  const double cpu_ms = std::chrono::duration<double, std::milli>(ce - cs).count();
  std::printf(
      "{\"mode\": \"%s\", \"batches\": %llu, \"mean_batch\": %.2f, \"max_batch\": %llu, "
      "\"threads\": %d, \"tables_per_thread\": %d, \"keys_per_table\": %d, \"failures\": %d, "
      "\"no_device_alloc_after_warmup\": %s, \"finish_ms\": {\"median\": %.4f, \"p90\": %.4f, \"p99\": %.4f, "
      "\"max\": %.4f, \"mean\": %.4f}, \"finish_over_2ms_by_table\": %s, \"host_sync\": \"%s\", "
      "\"addkey_ns_per_key\": %.2f, "
      "\"gpu_adapter\": {\"wall_ms\": %.2f, \"mkeys_s\": %.1f, \"tables_per_s\": %.0f}, "
      "\"cpu_oracle_same_threads\": {\"wall_ms\": %.2f, \"mkeys_s\": %.1f, \"ms_per_table\": %.3f}}\n",
      mode.c_str(), static_cast<unsigned long long>(nb), nb ? static_cast<double>(nj) / nb : 0.0,
      static_cast<unsigned long long>(mb), threads, tables, n, fails, no_alloc ? "true" : "false", pct(0.5), pct(0.9), pct(0.99),
      lat.empty() ? 0.0 : lat.back(), lat.empty() ? 0.0 : sum / lat.size(), slow.c_str(), hs ? hs : "default",
      add_ms * 1e6 / keys_timed, gpu_ms, keys_timed / (gpu_ms * 1e3), threads * tables / (gpu_ms * 1e-3),
      cpu_ms, keys_timed / (cpu_ms * 1e3), cpu_ms * threads / (threads * tables));
  if (fails == 0 && no_alloc) std::printf("OK concurrent builders\n");
  return fails == 0 && no_alloc ? 0 : 1;
}
