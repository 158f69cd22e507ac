// Diagnostic: the bench step (one batched build of T SSTable filters + one
// probe of Q lookups against F stacked filters) issued from a C++ host loop
// straight through the C ABI, as dLSM's C++ builder / Get threads would call
// it, with no Python between the calls.  Compares the per-step time with the
// Python-driven bench.py loop (whose kernel traces show ~10 us idle between
// the build call's last kernel and the probe call's first).  Timing only:
// parity is the tests' job.
//
//   step_loop [tables=16] [keys=1600000] [lookups=100000000] [steps=50] [warmup=10]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dlsm_bloom.h"

#define CK(x)                                                              \
  do {                                                                     \
    int _s = (x);                                                          \
    if (_s != 0) {                                                         \
      fprintf(stderr, "%s:%d: %s -> %d\n", __FILE__, __LINE__, #x, _s);    \
      return 1;                                                            \
    }                                                                      \
  } while (0)

// db_bench-shaped 20-byte keys: the value v as 16 decimal digits + "xxxx"
static void make_key(uint64_t v, uint8_t* out) {
  for (int i = 15; i >= 0; i--) {
    out[i] = static_cast<uint8_t>('0' + v % 10);
    v /= 10;
  }
  for (int i = 16; i < 20; i++) out[i] = 'x';
}

static uint64_t mix(uint64_t x) {  // splitmix64
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 16;
  const uint64_t N = argc > 2 ? strtoull(argv[2], nullptr, 10) : 1600000;
  const uint64_t Q = argc > 3 ? strtoull(argv[3], nullptr, 10) : 100000000;
  const int K = argc > 4 ? atoi(argv[4]) : 50;
  const int W = argc > 5 ? atoi(argv[5]) : 10;
  const int F = 8, bpk = 10;
  dlsm_ctx* ctx = nullptr;
  CK(dlsm_ctx_create(0, &ctx));
  // tables: table s <- v = TA * i + s (the first F also give the probed filter set)
  const int TA = T > F ? T : F;
  std::vector<uint8_t> h(N * 20);
  uint8_t* d_keys = nullptr;
  CK(hipMalloc(&d_keys, static_cast<size_t>(TA) * N * 20));
  for (int s = 0; s < TA; s++) {
    for (uint64_t i = 0; i < N; i++) make_key(static_cast<uint64_t>(TA) * i + s, &h[i * 20]);
    CK(hipMemcpy(d_keys + static_cast<size_t>(s) * N * 20, h.data(), N * 20, hipMemcpyHostToDevice));
  }
  uint64_t cap = 0;
  uint32_t lines = 0;
  CK(dlsm_bloom_full_size(N, bpk, &lines, &cap));
  cap = (cap + 15) / 16 * 16;
  uint8_t* d_out = nullptr;
  uint64_t* d_len = nullptr;
  CK(hipMalloc(&d_out, cap * TA));
  CK(hipMalloc(&d_len, sizeof(uint64_t) * TA));
  std::vector<dlsm_build_job> jobs(TA);
  for (int s = 0; s < TA; s++) {
    jobs[s].keys = dlsm_keyset{d_keys + static_cast<size_t>(s) * N * 20, nullptr, 20, 0, N};
    jobs[s].out = d_out + cap * s;
    jobs[s].out_cap = cap;
  }
  CK(dlsm_bloom_full_build_dev(ctx, jobs.data(), TA, bpk, d_len));
  CK(dlsm_ctx_sync(ctx));
  std::vector<uint64_t> lens(TA);
  CK(hipMemcpy(lens.data(), d_len, sizeof(uint64_t) * TA, hipMemcpyDeviceToHost));
  std::vector<const uint8_t*> fp(F);
  for (int f = 0; f < F; f++) fp[f] = d_out + cap * f;
  dlsm_filterset* fs = nullptr;
  CK(dlsm_filterset_create(ctx, fp.data(), lens.data(), F, 1, &fs));
  // lookups: hashed values over twice the key space (half of them absent)
  uint8_t* d_q = nullptr;
  uint8_t* d_mask = nullptr;
  CK(hipMalloc(&d_q, Q * 20));
  CK(hipMalloc(&d_mask, Q));
  {
    const uint64_t B = 1u << 22;
    std::vector<uint8_t> hq(B * 20);
    for (uint64_t b = 0; b < Q; b += B) {
      const uint64_t n = Q - b < B ? Q - b : B;
      for (uint64_t i = 0; i < n; i++) make_key(mix(b + i) % (2ull * TA * N), &hq[i * 20]);
      CK(hipMemcpy(d_q + b * 20, hq.data(), n * 20, hipMemcpyHostToDevice));
    }
  }
  const dlsm_keyset qk{d_q, nullptr, 20, 0, Q};
  auto step = [&]() -> int {
    CK(dlsm_bloom_full_build_dev(ctx, jobs.data(), T, bpk, d_len));
    CK(dlsm_bloom_full_probe_dev(ctx, fs, &qk, d_mask));
    return 0;
  };
  for (int i = 0; i < W; i++)
    if (step()) return 1;
  CK(dlsm_ctx_sync(ctx));
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < K; i++)
    if (step()) return 1;
  const auto t1 = std::chrono::steady_clock::now();
  CK(dlsm_ctx_sync(ctx));
  const auto t2 = std::chrono::steady_clock::now();
  const double ms = std::chrono::duration<double, std::milli>(t2 - t0).count() / K;
  const double enq = std::chrono::duration<double, std::milli>(t1 - t0).count() / K;
  printf("{\"driver\": \"c++ step loop\", \"tables\": %d, \"keys_per_table\": %llu, \"lookups\": %llu, "
         "\"steps\": %d, \"ms_per_step\": %.4f, \"host_enqueue_ms_per_step\": %.4f, \"mkeys_s\": %.1f}\n",
         T, static_cast<unsigned long long>(N), static_cast<unsigned long long>(Q), K, ms, enq,
         (static_cast<double>(T) * N + Q) / (ms * 1e3));
  dlsm_filterset_destroy(fs);
  dlsm_ctx_destroy(ctx);
  (void)hipFree(d_keys);
  (void)hipFree(d_out);
  (void)hipFree(d_len);
  (void)hipFree(d_q);
  (void)hipFree(d_mask);
  return 0;
}
