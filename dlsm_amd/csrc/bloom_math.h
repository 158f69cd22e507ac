// dlsm_amd/csrc/bloom_math.h -- arithmetic shared by the C-ABI host code and
// the gfx950 kernels.  Everything here is integer (u32 wraparound exactly as
// the reference); no floating point reaches an emitted byte except the one
// double product in the probe-count choice, evaluated on the host only.
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define DLSM_HD __host__ __device__ __forceinline__
#else
#define DLSM_HD inline
#endif

namespace dlsm {

// port/port_posix.h:301-306 (x86): the full-filter format's cache-line size.
constexpr uint32_t kCacheLineBytes = 64;
constexpr uint32_t kLineBits = kCacheLineBytes * 8;  // 512
// include/TimberSaw/filter_policy.h:26-28
constexpr uint32_t kBloomSeed = 0xbc9f1d34u;
constexpr uint32_t kHashM = 0xc6a4a793u;  // util/hash.cc:26

// util/hash.cc:22-62 on 4-byte words already loaded; `tail` holds the
// remaining 0-3 bytes (little-endian packed), `tail_len` their count.
DLSM_HD uint32_t hash_init(uint64_t n, uint32_t seed) {
  return seed ^ static_cast<uint32_t>(n * kHashM);
}
DLSM_HD uint32_t hash_word(uint32_t h, uint32_t w) {
  h += w;
  h *= kHashM;
  h ^= (h >> 16);
  return h;
}
// Tail bytes are sign-extended (util/hash.cc:49-59, static_cast<int8_t>).
DLSM_HD uint32_t hash_tail(uint32_t h, uint32_t tail, uint32_t tail_len) {
  switch (tail_len) {
    case 3:
      h += static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(tail >> 16))) << 16;
      [[fallthrough]];
    case 2:
      h += static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(tail >> 8))) << 8;
      [[fallthrough]];
    case 1:
      h += static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(tail)));
      h *= kHashM;
      h ^= (h >> 24);
      break;
    default:
      break;
  }
  return h;
}

// Host-side BloomHash over a byte pointer (adapters, tests).
inline uint32_t bloom_hash_host(const uint8_t* p, size_t n) {
  uint32_t h = hash_init(n, kBloomSeed);
  size_t i = 0;
  for (; i + 4 <= n; i += 4) {
    uint32_t w = uint32_t(p[i]) | (uint32_t(p[i + 1]) << 8) | (uint32_t(p[i + 2]) << 16) |
                 (uint32_t(p[i + 3]) << 24);
    h = hash_word(h, w);
  }
  uint32_t t = 0;
  for (size_t j = i; j < n; j++) t |= uint32_t(p[j]) << (8 * (j - i));
  return hash_tail(h, t, uint32_t(n - i));
}

// Exact u32 remainder by a run-time constant d >= 1.
// magic = floor((2^32-1)/d).  q = mulhi(h, magic) is q_true or q_true-1, so a
// single conditional subtract is exact for all h, d (checked exhaustively over
// adversarial d and random h in tests/test_host_abi.py).
DLSM_HD uint32_t fastmod_magic(uint32_t d) { return 0xffffffffu / d; }
DLSM_HD uint32_t fastmod(uint32_t h, uint32_t d, uint32_t magic) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t q = __umulhi(h, magic);
#else
  uint32_t q = static_cast<uint32_t>((static_cast<uint64_t>(h) * magic) >> 32);
#endif
  uint32_t r = h - q * d;
  return r >= d ? r - d : r;
}

// Quotient and remainder of h by d with the same magic (fastmod_magic(d)):
// q = mulhi(h, magic) is the true quotient or one less.
DLSM_HD uint32_t fastdivmod(uint32_t h, uint32_t d, uint32_t magic, uint32_t* rem) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t q = __umulhi(h, magic);
#else
  uint32_t q = static_cast<uint32_t>((static_cast<uint64_t>(h) * magic) >> 32);
#endif
  uint32_t r = h - q * d;
  if (r >= d) {
    r -= d;
    q++;
  }
  *rem = r;
  return q;
}

// util/bloom_impl.h:351-357 (full filter, int cast) -- host only (double).
inline int full_num_probes(int bits_per_key) {
  int k = static_cast<int>(bits_per_key * 0.69);
  if (k < 1) k = 1;
  if (k > 30) k = 30;
  return k;
}
// util/bloom.cc:16-21 (legacy policy, size_t cast).
inline int legacy_num_probes(int bits_per_key) {
  double p = bits_per_key * 0.69;
  size_t k = p < 0 ? 0 : static_cast<size_t>(p);
  if (k < 1) k = 1;
  if (k > 30) k = 30;
  return static_cast<int>(k);
}

// table/full_filter_block.cc:61-92 (GetTotalBitsForLocality + CalculateSpace),
// num_entry as the reference's `const int` (size_t -> int) and u32 products.
DLSM_HD uint32_t full_num_lines(uint64_t n_dedup, int bits_per_key, uint32_t* total_bits_out) {
  const int num_entry = static_cast<int>(static_cast<uint32_t>(n_dedup));
  uint32_t total_bits = 0, num_lines = 0;
  if (num_entry != 0) {
    uint32_t tb = static_cast<uint32_t>(num_entry) * static_cast<uint32_t>(bits_per_key);
    uint32_t nl = (tb + kLineBits - 1u) / kLineBits;
    if (nl % 2u == 0u) nl++;
    total_bits = nl * kLineBits;
    num_lines = total_bits / kLineBits;
  }
  if (total_bits_out) *total_bits_out = total_bits;
  return num_lines;
}
// Filter length written by Finish (full_filter_block.cc:134-139): total_bits/8 + 5.
DLSM_HD uint64_t full_filter_len(uint64_t n_dedup, int bits_per_key) {
  uint32_t tb;
  full_num_lines(n_dedup, bits_per_key, &tb);
  return static_cast<uint64_t>(tb / 8u) + 5u;
}

// util/bloom.cc:27-34: bits = max(n*bpk, 64) rounded up to whole bytes.
DLSM_HD uint64_t legacy_bits(uint64_t n, int bits_per_key) {
  uint64_t bits = n * static_cast<uint64_t>(static_cast<int64_t>(bits_per_key));
  if (bits < 64) bits = 64;
  return ((bits + 7) / 8) * 8;
}

// Rotate right 17 (util/bloom_impl.h:432, util/bloom.cc:46).
DLSM_HD uint32_t bloom_delta(uint32_t h) { return (h >> 17) | (h << 15); }

}  // namespace dlsm
