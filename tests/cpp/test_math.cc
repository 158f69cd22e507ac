// Host unit test of dlsm_amd/csrc/bloom_math.h (compiled with g++ by
// tests/test_host_abi.py).  Exhaustive-by-construction checks of the fastmod
// identity on adversarial divisors and the u32 sizing arithmetic.
#include <cstdio>
#include <cstdint>
#include <random>
#include "../../dlsm_amd/csrc/bloom_math.h"

int main() {
  using namespace dlsm;
  std::mt19937_64 rng(12345);
  uint64_t checks = 0;
  const uint32_t special_d[] = {1u, 2u, 3u, 5u, 7u, 31u, 511u, 512u, 513u, 3005u, 31251u, 65535u, 65536u,
                                65537u, 0x7fffffffu, 0x80000000u, 0x80000001u, 0xfffffffeu, 0xffffffffu};
  const uint32_t special_h[] = {0u, 1u, 2u, 0x7fffffffu, 0x80000000u, 0xfffffffeu, 0xffffffffu};
  for (uint32_t d : special_d) {
    const uint32_t m = fastmod_magic(d);
    for (uint32_t h : special_h) { if (fastmod(h, d, m) != h % d) { printf("FAIL d=%u h=%u\n", d, h); return 1; } checks++; }
    for (int i = 0; i < 200000; i++) { uint32_t h = (uint32_t)rng(); if (fastmod(h, d, m) != h % d) { printf("FAIL d=%u h=%u\n", d, h); return 1; } checks++; }
    // multiples of d and their neighbours
    for (uint64_t q = 0; q < 0x100000000ull; q += (0x100000000ull / 4096) | 1) {
      uint64_t x = (q / d) * d;
      for (int e = -1; e <= 1; e++) { uint64_t h = x + e; if (h > 0xffffffffull) continue;
        if (fastmod((uint32_t)h, d, m) != (uint32_t)h % d) { printf("FAIL d=%u h=%llu\n", d, (unsigned long long)h); return 1; } checks++; }
    }
  }
  for (int i = 0; i < 2000; i++) {
    uint32_t d = (uint32_t)rng() >> (rng() % 32); if (!d) d = 1;
    const uint32_t m = fastmod_magic(d);
    for (int j = 0; j < 2000; j++) { uint32_t h = (uint32_t)rng(); if (fastmod(h, d, m) != h % d) { printf("FAIL d=%u h=%u\n", d, h); return 1; } checks++; }
  }
  // sizing: L odd, covers n*bpk bits
  for (uint64_t n = 1; n < 200000; n += 7) {
    uint32_t tb; uint32_t L = full_num_lines(n, 10, &tb);
    if (L % 2 != 1 || (uint64_t)L * 512 < n * 10 || tb != L * 512) { printf("FAIL size n=%llu\n", (unsigned long long)n); return 1; }
  }
  if (full_num_lines(1600000, 10, nullptr) != 31251 || full_num_lines(153846, 10, nullptr) != 3005 ||
      full_num_lines(0, 10, nullptr) != 0 || full_filter_len(0, 10) != 5 || full_filter_len(1600000, 10) != 2000069) {
    printf("FAIL size constants\n"); return 1; }
  if (full_num_probes(10) != 6 || legacy_num_probes(10) != 6 || full_num_probes(0) != 1 || full_num_probes(100) != 30) {
    printf("FAIL probes\n"); return 1; }
  if (legacy_bits(0, 10) != 64 || legacy_bits(7, 10) != 72 || legacy_bits(1600000, 10) != 16000000) { printf("FAIL legacy bits\n"); return 1; }
  printf("OK %llu checks\n", (unsigned long long)checks);
  return 0;
}
