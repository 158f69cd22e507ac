// Diagnostic (host only; run by hand on a GPU box's host, results under
// profiles/): dlsm_bloom_hash_batch's rate on 20-byte keys by thread count,
// for a batch that stays in cache (64 Ki keys) and one streamed from DRAM
// (125.6 M keys: one bench step's build + probe keys, 2.5 GB).
//
//   g++ -O2 -std=c++17 -I include tests/diag/host_hash_rate.cc -L dlsm_amd/lib -ldlsm_bloom \
//       -Wl,-rpath,$PWD/dlsm_amd/lib -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -o tests/diag/hhr
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dlsm_bloom.h"

int main(int argc, char** argv) {
  const uint64_t big = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 125600000ull;
  for (uint64_t n : {uint64_t(65536), big}) {
    std::vector<uint8_t> k(n * 20 + 64);
    for (size_t i = 0; i < k.size(); i++) k[i] = static_cast<uint8_t>(i * 131 + (i >> 7));
    std::vector<uint32_t> out(n);
    dlsm_keyset ks{};
    ks.bytes = k.data();
    ks.n = n;
    ks.key_len = 20;
    const int reps = n < 100000 ? 2000 : 3;
    for (int th : {1, 2, 4, 8, 16, 0}) {
      dlsm_bloom_hash_batch(&ks, out.data(), th);
      const auto t0 = std::chrono::steady_clock::now();
      for (int r = 0; r < reps; r++) dlsm_bloom_hash_batch(&ks, out.data(), th);
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
      std::printf("{\"keys\": %llu, \"threads\": %d, \"ns_per_key\": %.3f, \"gkeys_s\": %.3f, \"key_GBs\": %.1f}\n",
                  static_cast<unsigned long long>(n), th, s / n * 1e9, n / s / 1e9, n * 20.0 / s / 1e9);
    }
  }
  return 0;
}
