// CPU microbenchmark of the adapter's AddKey (hash_in_addkey): the C ABI
// entry points the builder touches are stubbed here with malloc'd memory, so
// the loop runs without a GPU (diagnostic only; the real rate is measured by
// tests/cpp/concurrent_builders.cc on the GPU box).
//   g++ -std=c++17 -O2 -I include tests/diag/addkey_bench.cc -o /tmp/addkey_bench
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dlsm_bloom_adapter.hpp"

extern "C" {
int dlsm_bloom_full_num_probes(int) { return 6; }
int dlsm_ctx_host_buffer_claim(dlsm_ctx*, const void*) { return DLSM_E_BUSY; }
int dlsm_ctx_host_buffer_release(dlsm_ctx*, const void*) { return DLSM_OK; }
int dlsm_ctx_host_buffer(dlsm_ctx*, uint64_t, uint64_t, void**, uint64_t*) { return DLSM_E_ARG; }
int dlsm_host_pool_acquire(uint64_t min_bytes, void** out, uint64_t* cap) {
  *out = std::aligned_alloc(4096, (min_bytes + 4095) & ~uint64_t(4095));
  *cap = (min_bytes + 4095) & ~uint64_t(4095);
  return DLSM_OK;
}
int dlsm_host_pool_release(void* p) {
  std::free(p);
  return DLSM_OK;
}
int dlsm_ctx_get_option(dlsm_ctx*, int, uint64_t* v) {
  *v = 0;
  return DLSM_OK;
}
int dlsm_ctx_set_option(dlsm_ctx*, int, uint64_t) { return DLSM_OK; }
int dlsm_bloom_full_build(dlsm_ctx*, const dlsm_build_job*, int, int, uint64_t* len) {
  *len = 0;
  return DLSM_OK;
}
int dlsm_bloom_full_build_hashed(dlsm_ctx*, const dlsm_build_job* j, int, int, uint64_t* len) {
  // keep the staged hashes observable so the loop is not optimised away
  uint32_t x = 0;
  const uint32_t* h = reinterpret_cast<const uint32_t*>(j->keys.bytes);
  for (uint64_t i = 0; i < j->keys.n; i += 997) x ^= h[i];
  *len = x & 1;
  return DLSM_OK;
}
int dlsm_batcher_full_build(dlsm_batcher*, const dlsm_build_job*, int, uint64_t*) { return DLSM_E_ARG; }
int dlsm_batcher_full_build_hashed(dlsm_batcher*, const dlsm_build_job*, int, uint64_t*) { return DLSM_E_ARG; }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 153846;
  const int tables = argc > 2 ? std::atoi(argv[2]) : 40;
  std::vector<char> keys(static_cast<size_t>(n) * 20);
  for (int i = 0; i < n; i++) std::snprintf(&keys[20 * static_cast<size_t>(i)], 21, "%020d", i * 7 + 1);
  std::vector<char> slot(1 << 20);
  dlsm_adapter::FilterSlot mr{slot.data(), slot.size()};
  dlsm_adapter::BuilderOptions opt;
  opt.hash_in_addkey = true;
  dlsm_adapter::FullFilterBlockBuilder b(&mr, 10, reinterpret_cast<dlsm_ctx*>(&slot), opt);
  double best = 1e30;
  uint64_t sink = 0;
  for (int t = 0; t < tables; t++) {
    b.RestartBlock(0);
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) b.AddKey(dlsm_adapter::Slice(&keys[20 * static_cast<size_t>(i)], 20));
    const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
    best = ns < best ? ns : best;
    b.Finish();
    sink += b.result.size();
  }
  std::printf("{\"addkey_ns_per_key_best\": %.3f, \"keys\": %d, \"tables\": %d, \"sink\": %llu}\n", best / n, n,
              tables, static_cast<unsigned long long>(sink));
  return 0;
}
