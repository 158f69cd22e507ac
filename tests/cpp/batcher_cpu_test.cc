// The batcher's queue logic (dlsm_amd/csrc/batcher.hip) on the CPU, under
// ThreadSanitizer: the C-ABI build calls it makes are stubbed here, so no GPU
// is needed.  Shape that broke round 3: two executors with
// a gathering window, bursty submitters, and queues that drain to empty while
// an executor still waits in its window.  Also checks that one invalid job
// fails only its own caller (the batch is re-run job by job), that the
// DLSM_BATCH_EXACT flag reaches the executor's context, and that a too-small
// slot fails only its job.
//
//   g++ -std=c++17 -O1 -g -fsanitize=thread -pthread -I include -x c++ \
//       dlsm_amd/csrc/batcher.hip tests/cpp/batcher_cpu_test.cc
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "dlsm_bloom.h"

// ---- stubbed ABI: a "build" sleeps a little and reports a length that
// encodes what the executor's context was told --------------------------------
struct dlsm_ctx {
  std::atomic<int> exact{0};
};
static std::atomic<int> g_calls{0}, g_ctx_live{0};

extern "C" {
int dlsm_ctx_create(int, dlsm_ctx** out) {
  *out = new dlsm_ctx();
  g_ctx_live++;
  return DLSM_OK;
}
int dlsm_ctx_destroy(dlsm_ctx* c) {
  delete c;
  g_ctx_live--;
  return DLSM_OK;
}
int dlsm_ctx_set_option(dlsm_ctx* c, int opt, uint64_t v) {
  if (opt == DLSM_OPT_BUILD_EXACT) c->exact = static_cast<int>(v);
  return DLSM_OK;
}
static int stub_build(dlsm_ctx* c, const dlsm_build_job* jobs, int n, uint64_t* lens, uint64_t tag) {
  g_calls++;
  std::this_thread::sleep_for(std::chrono::microseconds(150));
  int st = DLSM_OK;
  for (int j = 0; j < n; j++)
    if (jobs[j].keys.key_len == 3) return DLSM_E_ARG;  // the library's validation: the whole call fails
  for (int j = 0; j < n; j++) {
    if (jobs[j].out_cap < jobs[j].keys.n) {
      lens[j] = 0;
      st = DLSM_E_CAPACITY;
      continue;
    }
    lens[j] = jobs[j].keys.n * 10 + static_cast<uint64_t>(c->exact) + tag;
  }
  return st;
}
int dlsm_bloom_full_build(dlsm_ctx* c, const dlsm_build_job* jobs, int n, int, uint64_t* lens) {
  return stub_build(c, jobs, n, lens, 0);
}
int dlsm_bloom_full_build_hashed(dlsm_ctx* c, const dlsm_build_job* jobs, int n, int, uint64_t* lens) {
  return stub_build(c, jobs, n, lens, 1000000);
}
}  // extern "C"

int main() {
  std::atomic<int> failures{0};
  for (uint32_t window : {0u, 50u, 400u}) {
    dlsm_batcher* b = nullptr;
    if (dlsm_batcher_create(0, 3, window, 8, &b) != DLSM_OK) {
      std::printf("FAIL create\n");
      return 1;
    }
    const int T = 12, per = 40;
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) {
      th.emplace_back([&, t] {
        std::mt19937 rng(1234 + t);
        for (int i = 0; i < per; i++) {
          dlsm_build_job job{};
          const uint64_t n = 1 + rng() % 1000;
          job.keys.n = n;
          job.keys.key_len = (t == 3 && i % 7 == 0) ? 3 : 20;  // an invalid job now and then
          job.out_cap = (t == 5 && i % 5 == 0) ? n - 1 : n;    // a too-small slot now and then
          int flags = 0;
          if (i % 3 == 0) flags |= DLSM_BATCH_EXACT;
          if (t % 2) flags |= DLSM_BATCH_HASHED;
          uint64_t len = 12345;
          const int st = dlsm_batcher_submit(b, &job, 10, flags, &len);
          int want_st = DLSM_OK;
          uint64_t want_len = n * 10 + ((flags & DLSM_BATCH_EXACT) ? 1 : 0) + ((flags & DLSM_BATCH_HASHED) ? 1000000 : 0);
          if (job.keys.key_len == 3) {
            want_st = DLSM_E_ARG;
            want_len = 0;
          } else if (job.out_cap < n) {
            want_st = DLSM_E_CAPACITY;
            want_len = 0;
          }
          if (st != want_st || len != want_len) {
            std::printf("FAIL window %u thread %d job %d: status %d (want %d) len %llu (want %llu)\n", window, t, i,
                        st, want_st, static_cast<unsigned long long>(len), static_cast<unsigned long long>(want_len));
            failures++;
          }
          // bursts: a pause after every few submissions lets the queue drain
          // to empty while other executors wait in their windows
          if (i % 4 == 3) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 900));
        }
      });
    }
    for (auto& x : th) x.join();
    uint64_t nb = 0, nj = 0, mb = 0;
    dlsm_batcher_stats(b, &nb, &nj, &mb);
    if (nj != static_cast<uint64_t>(T) * per || nb == 0 || nb > nj || mb > 8) {
      std::printf("FAIL stats window %u: batches %llu jobs %llu max %llu\n", window, (unsigned long long)nb,
                  (unsigned long long)nj, (unsigned long long)mb);
      failures++;
    }
    dlsm_batcher_destroy(b);
  }
  if (g_ctx_live != 0) {
    std::printf("FAIL %d contexts leaked\n", g_ctx_live.load());
    failures++;
  }
  if (failures) return 1;
  std::printf("OK batcher cpu (%d stub builds)\n", g_calls.load());
  return 0;
}
