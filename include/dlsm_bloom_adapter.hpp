// dlsm_bloom_adapter.hpp -- header-only C++ mirror of dLSM's filter classes
// over the C ABI (dlsm_bloom.h).  Same class and method names, argument
// meaning and call order as the reference, so a TableBuilder / Table / DB
// can swap them in (INTEGRATION.md shows the reference-side edit):
//
//   FilterPolicy            include/TimberSaw/filter_policy.h:31-55
//       the abstract interface (virtual Name / CreateFilter / KeyMayMatch)
//   BloomFilterPolicy       util/bloom.cc:14-91 (: FilterPolicy),
//       NewBloomFilterPolicy util/bloom.cc:89-91
//   InternalFilterPolicy    db/dbformat.h:399-408, db/dbformat.cc:93-109
//       (: FilterPolicy) -- internal keys, hashed as ExtractUserKey(key)
//   FullFilterBlockBuilder  table/full_filter_block.h:33-70
//       (RestartBlock AddKey*)* Finish; Reset; Move_buffer; public `result`
//   FullFilterBlockReader   table/full_filter_block.h:71-94
//       ctor parses metadata; KeyMayMatch; + KeysMayMatch (batch)
//   FilterBlockBuilder      table/filter_block.h:34-68 (legacy 2 KiB framing)
//       StartBlock AddKey* ... Finish; public `result`
//   FilterBlockReader       table/filter_block.h:70-85
//       KeyMayMatch(block_offset, key) + KeysMayMatch (batch)
//
// Host types.  By default the header declares its own Slice and FilterPolicy
// with the reference's surface.  Inside the reference tree, define
// DLSM_ADAPTER_HOST_NAMESPACE to the host's namespace (TimberSaw) before
// including it: the adapter then uses TimberSaw::Slice and derives from
// TimberSaw::FilterPolicy, so a BloomFilterPolicy / InternalFilterPolicy from
// here can be stored in Options::filter_policy (options.h:185-187).
//
// No exceptions and no RTTI (the reference builds with -fno-exceptions
// -fno-rtti): failures are reported through status().
//
// Where the work runs.  Filter builds (Finish, CreateFilter) and batch probes
// (KeysMayMatch) run on the GPU behind the ABI.  A single-key KeyMayMatch --
// Table::InternalGet's per-Get call (table/table.cc:357), ~38 ns on the
// reference's CPU -- is answered on the host from the filter bytes: one GPU
// round trip per key would cost microseconds.  A GPU call that fails (device
// error, out of memory, no device) is re-run by the reference's own host
// loop, so no caller ever receives a 0-byte or partial filter; every such
// re-run is counted (dlsm_fallback_stats) and the parity tests assert the
// count stays 0 on their GPU runs.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#if defined(__x86_64__)
#include <immintrin.h>
#endif
#include <string>
#include <vector>

#include "dlsm_bloom.h"

namespace dlsm_adapter {

#ifdef DLSM_ADAPTER_HOST_NAMESPACE
using Slice = ::DLSM_ADAPTER_HOST_NAMESPACE::Slice;
using FilterPolicy = ::DLSM_ADAPTER_HOST_NAMESPACE::FilterPolicy;
#else
// Byte view with the reference Slice's surface used on this path
// (include/TimberSaw/slice.h:27-103): data/size/Reset/append.
class Slice {
 public:
  Slice() : data_(""), size_(0) {}
  Slice(const char* d, size_t n) : data_(d), size_(n) {}
  Slice(const std::string& s) : data_(s.data()), size_(s.size()) {}  // NOLINT
  const char* data() const { return data_; }
  size_t size() const { return size_; }
  bool empty() const { return size_ == 0; }
  void Reset(const char* d, size_t n) {
    data_ = d;
    size_ = n;
  }
  // Unchecked, like the reference (slice.h:93-97).
  void append(const char* p, size_t n) {
    memcpy(const_cast<char*>(data_) + size_, p, n);
    size_ += n;
  }
  std::string ToString() const { return std::string(data_, size_); }

 private:
  const char* data_;
  size_t size_;
};

// include/TimberSaw/filter_policy.h:31-55
class FilterPolicy {
 public:
  virtual ~FilterPolicy() {}
  virtual const char* Name() const = 0;
  // Append a filter summarising keys[0, n) to *dst (initial contents kept).
  virtual void CreateFilter(const Slice* keys, int n, Slice* dst) const = 0;
  virtual bool KeyMayMatch(const Slice& key, const Slice& filter) const = 0;
};
#endif

// db/dbformat.h:374-377 (asserts internal_key.size() >= 8).
inline Slice ExtractUserKey(const Slice& internal_key) {
  return Slice(internal_key.data(), internal_key.size() >= DLSM_INTERNAL_KEY_TRAILER
                                        ? internal_key.size() - DLSM_INTERNAL_KEY_TRAILER
                                        : 0);
}

// BloomHash(key) = Hash(key, n, 0xbc9f1d34) (include/TimberSaw/filter_policy.h:
// 26-28, util/hash.cc:22-62): MurmurHash1-style over little-endian 4-byte
// words, the 1-3 tail bytes sign-extended.  Inline so AddKey can hash on the
// host exactly as the reference's AddKey does (the library's
// dlsm_bloom_hash gives the same value; tests compare them).
inline uint32_t BloomHash(const char* data, size_t n) {
  const uint32_t m = 0xc6a4a793u;
  uint32_t h = 0xbc9f1d34u ^ static_cast<uint32_t>(n * m);
  const unsigned char* p = reinterpret_cast<const unsigned char*>(data);
  if (n == 20) {  // db_bench keys (key_size 20): five words, no tail
    uint32_t w[5];
    std::memcpy(w, p, 20);
    for (int j = 0; j < 5; j++) {
      h += w[j];
      h *= m;
      h ^= (h >> 16);
    }
    return h;
  }
  size_t i = 0;
  for (; i + 4 <= n; i += 4) {
    uint32_t w;
    std::memcpy(&w, p + i, 4);  // x86 / gfx hosts: little-endian, like DecodeFixed32
    h += w;
    h *= m;
    h ^= (h >> 16);
  }
  const auto sx = [](unsigned char c) { return static_cast<uint32_t>(static_cast<int32_t>(static_cast<int8_t>(c))); };
  switch (n - i) {
    case 3:
      h += sx(p[i + 2]) << 16;
      [[fallthrough]];
    case 2:
      h += sx(p[i + 1]) << 8;
      [[fallthrough]];
    case 1:
      h += sx(p[i]);
      h *= m;
      h ^= (h >> 24);
      break;
    default:
      break;
  }
  return h;
}

// BloomHash of four 20-byte keys at p, p+20, p+40, p+60 (four independent
// chains the CPU overlaps; same values as BloomHash).
inline void BloomHash20x4(const char* p, uint32_t* out) {
  const uint32_t m = 0xc6a4a793u;
  uint32_t w[20];
  std::memcpy(w, p, 80);
  uint32_t h0 = 0xbc9f1d34u ^ static_cast<uint32_t>(20u * m), h1 = h0, h2 = h0, h3 = h0;
  for (int j = 0; j < 5; j++) {
    h0 += w[j];
    h1 += w[5 + j];
    h2 += w[10 + j];
    h3 += w[15 + j];
    h0 *= m;
    h1 *= m;
    h2 *= m;
    h3 *= m;
    h0 ^= h0 >> 16;
    h1 ^= h1 >> 16;
    h2 ^= h2 >> 16;
    h3 ^= h3 >> 16;
  }
  out[0] = h0;
  out[1] = h1;
  out[2] = h2;
  out[3] = h3;
}

#if defined(__x86_64__) && (defined(__GNUC__) || defined(__clang__))
// BloomHash of sixteen 20-byte keys at p .. p+300 with AVX-512: the 80 words
// load as five 16-lane vectors, word j of key k (dword 5k + j) is gathered
// across them with two-source permutes, and the five hash rounds run on all
// 16 keys at once.  Same values as BloomHash; used when the CPU has AVX-512F
// (dlsm_adapter::HasAvx512).
__attribute__((target("avx512f"))) inline void BloomHash20x16(const char* p, uint32_t* out) {
  const __m512i v0 = _mm512_loadu_si512(p), v1 = _mm512_loadu_si512(p + 64), v2 = _mm512_loadu_si512(p + 128),
                v3 = _mm512_loadu_si512(p + 192), v4 = _mm512_loadu_si512(p + 256);
  const __m512i k = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
  const __m512i k5 = _mm512_mullo_epi32(k, _mm512_set1_epi32(5));
  const __m512i m = _mm512_set1_epi32(static_cast<int>(0xc6a4a793u));
  __m512i h = _mm512_set1_epi32(static_cast<int>(0xbc9f1d34u ^ (20u * 0xc6a4a793u)));
  for (int j = 0; j < 5; j++) {
    const __m512i d = _mm512_add_epi32(k5, _mm512_set1_epi32(j));  // dword index 5k + j, 0..79
    const __m512i lo = _mm512_permutex2var_epi32(v0, d, v1);          // d in [0, 32)
    const __m512i mid = _mm512_permutex2var_epi32(v2, d, v3);         // d in [32, 64)
    const __m512i hi = _mm512_permutexvar_epi32(d, v4);               // d in [64, 80)
    const __mmask16 ge32 = _mm512_cmpge_epu32_mask(d, _mm512_set1_epi32(32));
    const __mmask16 ge64 = _mm512_cmpge_epu32_mask(d, _mm512_set1_epi32(64));
    const __m512i w = _mm512_mask_blend_epi32(ge64, _mm512_mask_blend_epi32(ge32, lo, mid), hi);
    h = _mm512_add_epi32(h, w);
    h = _mm512_mullo_epi32(h, m);
    h = _mm512_xor_si512(h, _mm512_srli_epi32(h, 16));
  }
  _mm512_storeu_si512(out, h);
}
inline bool HasAvx512() {
  static const bool has = __builtin_cpu_supports("avx512f");
  return has;
}
// AddKey's consecutive-duplicate drop (full_filter_block.cc:45-48) over n
// hashes, n a multiple of 16: each vector is compared with itself shifted by
// one hash (the previous hash in front), the kept lanes are compressed
// together in a register and stored.  Writes up to 64 bytes at out + 4*kept
// (the caller leaves that much room); returns the number kept.
__attribute__((target("avx512f"))) inline size_t DedupStore16(const uint32_t* h, size_t n, uint32_t last,
                                                              bool keep_first, uint8_t* out) {
  size_t kept = 0;
  __m512i prev = _mm512_set1_epi32(static_cast<int>(last));
  for (size_t j = 0; j < n; j += 16) {
    const __m512i v = _mm512_loadu_si512(h + j);
    const __m512i pv = _mm512_alignr_epi32(v, prev, 15);  // [prev[15], v[0] .. v[14]]
    __mmask16 keep = _mm512_cmpneq_epu32_mask(v, pv);
    if (keep_first && j == 0) keep = static_cast<__mmask16>(keep | 1u);
    _mm512_storeu_si512(out + 4 * kept, _mm512_maskz_compress_epi32(keep, v));
    kept += static_cast<size_t>(__builtin_popcount(keep));
    prev = v;
  }
  return kept;
}
#else
inline void BloomHash20x16(const char* p, uint32_t* out) {
  for (int q = 0; q < 4; q++) BloomHash20x4(p + 80 * q, out + 4 * q);
}
inline bool HasAvx512() { return false; }
inline size_t DedupStore16(const uint32_t*, size_t, uint32_t, bool, uint8_t*) { return 0; }
#endif


// ---------------------------------------------------------------------------
// Host forms of the filter arithmetic.  Product code, not the oracle: the
// single-key probes answer from these, and a build the GPU could not run
// falls back to them (the reference's own loops, restated).
// ---------------------------------------------------------------------------
namespace host {

inline void PutFixed32(char* p, uint32_t v) {  // util/coding.h:130-142 (little-endian)
  p[0] = static_cast<char>(v);
  p[1] = static_cast<char>(v >> 8);
  p[2] = static_cast<char>(v >> 16);
  p[3] = static_cast<char>(v >> 24);
}
inline uint32_t GetFixed32(const char* p) {  // util/coding.h:184-193
  const unsigned char* u = reinterpret_cast<const unsigned char*>(p);
  return uint32_t(u[0]) | (uint32_t(u[1]) << 8) | (uint32_t(u[2]) << 16) | (uint32_t(u[3]) << 24);
}

// LegacyLocalityBloomImpl<false>::AddHash (util/bloom_impl.h:427-443) with
// 64-byte lines: line h % L, then k bits of that line at h, h + delta, ...
inline void AddHash(uint32_t h, uint32_t num_lines, int k, char* data) {
  char* line = data + (static_cast<uint64_t>(h % num_lines) << 6);
  const uint32_t delta = (h >> 17) | (h << 15);
  for (int i = 0; i < k; i++) {
    const uint32_t bitpos = h & 511u;
    line[bitpos >> 3] = static_cast<char>(line[bitpos >> 3] | (1 << (bitpos & 7)));
    h += delta;
  }
}

// FullFilterBlockBuilder::Finish (table/full_filter_block.cc:93-141) over the
// hashes h[0, n): CalculateSpace (:61-92) of the consecutive-distinct count,
// AddHash per kept hash, then the k byte and Fixed32 line count.  dedup drops
// a hash equal to its predecessor first (AddKey's check, :45-48; the
// reference's hash_entries_ are already deduplicated).  Writes every byte of
// the filter, zeros included (the reference ORs into a zeroed slot).  Returns
// the filter length, or 0 when it does not fit in cap bytes.
inline uint64_t FullFilterFromHashes(const uint32_t* h, size_t n, int bits_per_key, char* out, size_t cap,
                                     bool dedup) {
  uint64_t kept = n;
  if (dedup) {
    kept = 0;
    for (size_t i = 0; i < n; i++) kept += (i == 0 || h[i] != h[i - 1]) ? 1 : 0;
  }
  uint32_t L = 0;
  uint64_t len = 0;
  dlsm_bloom_full_size(kept, bits_per_key, &L, &len);
  if (len > cap || !out) return 0;
  const int k = dlsm_bloom_full_num_probes(bits_per_key);
  std::memset(out, 0, static_cast<size_t>(L) * 64);
  if (L)
    for (size_t i = 0; i < n; i++)
      if (!dedup || i == 0 || h[i] != h[i - 1]) AddHash(h[i], L, k, out);
  out[static_cast<size_t>(L) * 64] = static_cast<char>(k);
  PutFixed32(out + static_cast<size_t>(L) * 64 + 1, L);
  return len;
}

// A one-line filter with every bit set ([64 x 0xff][k][Fixed32 1]): the
// reference reader accepts it (full_filter_block.cc:241-249) and every
// KeyMayMatch answers true -- never a false negative.  Finish emits it when
// the slot cannot hold the real filter (the reference only asserts there,
// :103, and writes past the slot in release builds).  Returns 69, or 0 if
// cap < 69.
constexpr size_t kMatchAllLen = 64 + 5;
inline uint64_t MatchAllFilter(int bits_per_key, char* out, size_t cap) {
  if (cap < kMatchAllLen || !out) return 0;
  std::memset(out, 0xff, 64);
  out[64] = static_cast<char>(dlsm_bloom_full_num_probes(bits_per_key));
  PutFixed32(out + 65, 1);
  return kMatchAllLen;
}

// The parsed metadata of a full filter (FullFilterBlockReader ctor,
// full_filter_block.cc:186-252, via dlsm_bloom_full_parse: DLSM_E_CORRUPT
// where the reference exit(1)s or could not probe).
struct FullFilterMeta {
  int status = DLSM_E_CORRUPT;
  int k = 0;
  uint32_t num_lines = 0;
  int log2_line = 0;
};
inline FullFilterMeta ParseFull(const char* data, size_t len) {
  FullFilterMeta m;
  m.status = dlsm_bloom_full_parse(reinterpret_cast<const uint8_t*>(data), len, &m.k, &m.num_lines, &m.log2_line);
  return m;
}

// FullFilterBlockReader::KeyMayMatch's probe (full_filter_block.cc:269-284 ->
// PrepareHashMayMatch / HashMayMatchPrepared, util/bloom_impl.h:445-481) of
// hash h: line h % L of 2^log2_line bytes, k bits at h, h + delta, ...
inline bool FullHashMayMatch(const char* data, const FullFilterMeta& m, uint32_t h) {
  const char* line = data + (static_cast<uint64_t>(h % m.num_lines) << m.log2_line);
  const uint32_t mask = (1u << (m.log2_line + 3)) - 1u;
  const uint32_t delta = (h >> 17) | (h << 15);
  for (int i = 0; i < m.k; i++) {
    const uint32_t bitpos = h & mask;
    if ((line[bitpos >> 3] & (1 << (bitpos & 7))) == 0) return false;
    h += delta;
  }
  return true;
}

// BloomFilterPolicy's k (util/bloom.cc:16-21).
inline int LegacyNumProbes(int bits_per_key) {
  int k = static_cast<int>(bits_per_key * 0.69);
  return k < 1 ? 1 : (k > 30 ? 30 : k);
}

// BloomFilterPolicy::CreateFilter (util/bloom.cc:25-55): the filter of
// keys[0, n) (each hashed as its first size - suffix_len bytes: the user key
// of an internal key) into out[0, bytes + 1).  Zeroes the bit array first
// (the reference ORs into whatever the buffer holds).  Returns bytes + 1.
inline uint64_t LegacyCreateFilter(const Slice* keys, int n, int bits_per_key, uint32_t suffix_len, char* out) {
  size_t bits = static_cast<size_t>(n < 0 ? 0 : n) * static_cast<size_t>(bits_per_key);
  if (bits < 64) bits = 64;
  const size_t bytes = (bits + 7) / 8;
  bits = bytes * 8;
  const int k = LegacyNumProbes(bits_per_key);
  std::memset(out, 0, bytes);
  for (int i = 0; i < n; i++) {
    const size_t len = keys[i].size() >= suffix_len ? keys[i].size() - suffix_len : 0;
    uint32_t h = BloomHash(keys[i].data(), len);
    const uint32_t delta = (h >> 17) | (h << 15);
    for (int j = 0; j < k; j++) {
      const uint32_t bitpos = static_cast<uint32_t>(h % bits);
      out[bitpos / 8] = static_cast<char>(out[bitpos / 8] | (1 << (bitpos % 8)));
      h += delta;
    }
  }
  out[bytes] = static_cast<char>(k);
  return bytes + 1;
}

// BloomFilterPolicy::KeyMayMatch (util/bloom.cc:57-81): len < 2 -> false; the
// stored k read as char -> size_t, > 30 (negative included) -> true.
inline bool LegacyKeyMayMatch(const char* key, size_t key_len, const char* filter, size_t len) {
  if (len < 2) return false;
  const size_t bits = (len - 1) * 8;
  const size_t k = static_cast<size_t>(static_cast<signed char>(filter[len - 1]));
  if (k > 30) return true;
  uint32_t h = BloomHash(key, key_len);
  const uint32_t delta = (h >> 17) | (h << 15);
  for (size_t j = 0; j < k; j++) {
    const uint32_t bitpos = static_cast<uint32_t>(h % bits);
    if ((filter[bitpos / 8] & (1 << (bitpos % 8))) == 0) return false;
    h += delta;
  }
  return true;
}

// FilterBlockReader ctor + KeyMayMatch (table/filter_block.cc:114-142) with
// the legacy policy: the filter of the data block at block_offset, or true
// ("errors are treated as potential matches").
inline bool FilterBlockKeyMayMatch(const char* contents, size_t n, uint64_t block_offset, const char* key,
                                   size_t key_len) {
  if (n < 5) return true;
  const unsigned base_lg = static_cast<unsigned>(static_cast<int>(static_cast<signed char>(contents[n - 1])));
  const uint32_t last_word = GetFixed32(contents + n - 5);
  if (last_word > n - 5) return true;
  const char* offset = contents + last_word;
  const uint64_t num = (n - 5 - last_word) / 4;
  const uint64_t index = block_offset >> (base_lg & 63u);  // x86 shift count
  if (index < num) {
    const uint32_t start = GetFixed32(offset + index * 4);
    const uint32_t limit = GetFixed32(offset + index * 4 + 4);
    if (start <= limit && limit <= last_word) return LegacyKeyMayMatch(key, key_len, contents + start, limit - start);
    if (start == limit) return false;
  }
  return true;
}

}  // namespace host

// Stand-in for the ibv_mr the reference builder borrows: the filter slot.
// (The reference-signature constructor below takes any type with `addr` and
// `length` -- ibv_mr itself binds as-is.)
struct FilterSlot {
  void* addr;
  size_t length;
};

// The calling thread's context (dlsm_thread_ctx): created by the library on
// the thread's first builder, on the i-th asking thread's device i mod the
// device count; nullptr if no device is visible (Finish then reports it).
inline dlsm_ctx* ThreadContext() {
  dlsm_ctx* c = nullptr;
  return dlsm_thread_ctx(&c) == DLSM_OK ? c : nullptr;
}

// std::allocator's contract over the library's page-locked host pool
// (dlsm_host_pool_*): a std::vector<uint32_t, PinnedAllocator<uint32_t>> is
// the reference's hash_entries_ with its storage in DMA-able memory, so
// Finish's upload of the hashes runs at the link rate instead of through the
// runtime's pageable staging.  When the pool cannot page-lock more memory
// (memlock limit, pinned-memory pressure) the storage comes from malloc
// instead: the upload is then staged by the runtime, slower but the same
// bytes.  deallocate tells the two apart by the pool's own answer (it refuses
// a pointer it did not hand out).  Only an exhausted heap aborts, as operator
// new does under -fno-exceptions.
template <class T>
struct PinnedAllocator {
  using value_type = T;
  PinnedAllocator() = default;
  template <class U>
  PinnedAllocator(const PinnedAllocator<U>&) {}  // NOLINT
  T* allocate(size_t n) {
    void* p = nullptr;
    uint64_t cap = 0;
    if (dlsm_host_pool_acquire(n * sizeof(T), &p, &cap) == DLSM_OK && p) return static_cast<T*>(p);
    p = std::malloc(n * sizeof(T) > 0 ? n * sizeof(T) : 1);
    if (!p) std::abort();
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t) {
    if (dlsm_host_pool_release(p) != DLSM_OK) std::free(p);
  }
  friend bool operator==(const PinnedAllocator&, const PinnedAllocator&) { return true; }
  friend bool operator!=(const PinnedAllocator&, const PinnedAllocator&) { return false; }
};

// Key staging in page-locked host memory: AddKey writes the keys where
// Finish's H2D DMA reads them.  The first builder on a context claims the
// context's own buffer (dlsm_ctx_host_buffer_claim), so builders created one
// after another per SSTable reuse it and allocate nothing after the first
// table; a builder that finds it held by another live builder on the same
// context stages into a private pinned buffer instead of sharing bytes.
class PinnedBytes {
 public:
  explicit PinnedBytes(dlsm_ctx* ctx) : ctx_(ctx) {}
  PinnedBytes(const PinnedBytes&) = delete;
  PinnedBytes& operator=(const PinnedBytes&) = delete;
  ~PinnedBytes() {
    if (shared_) dlsm_ctx_host_buffer_release(ctx_, this);
    else if (p_) free_private(p_);
  }
  bool append(const char* d, size_t n) {
    if (size_ + n > cap_ && !grow(size_ + n)) return false;
    memcpy(p_ + size_, d, n);
    size_ += n;
    return true;
  }
  // Room for n more bytes at the end (nullptr if it cannot grow); advance()
  // then keeps any prefix of them -- AddKey's branch-free hash staging.
  uint8_t* tail(size_t n) {
    if (size_ + n > cap_ && !grow(size_ + n)) return nullptr;
    return p_ + size_;
  }
  void advance(size_t n) { size_ += n; }
  void clear() { size_ = 0; }
  const uint8_t* data() const { return p_ ? p_ : reinterpret_cast<const uint8_t*>(""); }
  size_t size() const { return size_; }
  bool shared() const { return shared_; }

 private:
  bool grow(size_t need) {
    if (!decided_) {
      decided_ = true;
      shared_ = dlsm_ctx_host_buffer_claim(ctx_, this) == DLSM_OK;
    }
    void* q = nullptr;
    if (shared_) {
      uint64_t c = 0;
      if (dlsm_ctx_host_buffer(ctx_, need, size_, &q, &c) != DLSM_OK) return false;
      p_ = static_cast<uint8_t*>(q);
      cap_ = c;
      return true;
    }
    // a private buffer from the library's page-locked pool (builders created
    // per SSTable recycle them: no page-locking after the first tables); when
    // nothing more can be page-locked, from the heap (a slower upload, the
    // same bytes)
    uint64_t c = 0;
    size_t want = need > 2 * cap_ ? need : 2 * cap_;
    if (want < (size_t(1) << 20)) want = size_t(1) << 20;
    if (dlsm_host_pool_acquire(want, &q, &c) != DLSM_OK || !q) {
      q = std::malloc(want);
      if (!q) return false;
      c = want;
    }
    if (size_) memcpy(q, p_, size_);
    if (p_) free_private(p_);
    p_ = static_cast<uint8_t*>(q);
    cap_ = c;
    return true;
  }
  static void free_private(void* p) {
    if (dlsm_host_pool_release(p) != DLSM_OK) std::free(p);  // the pool refuses what it did not hand out
  }
  dlsm_ctx* ctx_;
  uint8_t* p_ = nullptr;
  size_t size_ = 0, cap_ = 0;
  bool decided_ = false, shared_ = false;
};

// How a builder hands its table to the GPU at Finish.
//  * ctx only: its own context, one synchronous build per table;
//  * batcher: the device's submission queue (dlsm_batcher): concurrent
//    Finish calls of many builder threads become one batched build;
//  * hash_in_addkey: AddKey's keys are hashed with BloomHash on the host
//    (in blocks of 256: independent chains overlap) and a hash equal to the
//    previous one is dropped -- the reference's own AddKey
//    (full_filter_block.cc:39-49) -- so Finish moves 4 bytes per distinct
//    key over PCIe instead of the key bytes, and the GPU builds from the
//    hashes (dlsm_bloom_full_build_hashed).  Same filter bytes either way.
struct BuilderOptions {
  dlsm_batcher* batcher = nullptr;
  bool hash_in_addkey = false;
};

class FullFilterBlockBuilder {
 public:
  // The reference's signature, table/full_filter_block.h:35 --
  // FullFilterBlockBuilder(ibv_mr* mr, int bloombits_per_key): `mr` is any
  // memory-region type with `addr` and `length` (ibv_mr binds as-is), the
  // context is the calling thread's (dlsm_thread_ctx).  AddKey is the
  // reference's own (full_filter_block.cc:39-49): BloomHash per key into
  // hash_entries_, a hash equal to the last one dropped; Finish replaces only
  // the scatter loop (:104-108): hash_entries_ (4 B per distinct key) goes to
  // the GPU, and the kernels write the filter -- every byte, then the k byte
  // and Fixed32 line count -- straight into the slot when it is page-locked
  // (dlsm_host_register the RDMA chunk once), else through staging.
  template <class MR>
  FullFilterBlockBuilder(MR* mr, int bits_per_key)
      : slot_{mr->addr, static_cast<size_t>(mr->length)}, local_mr_(&slot_), bits_per_key_(bits_per_key),
        num_probes_(dlsm_bloom_full_num_probes(bits_per_key)), ctx_(ThreadContext()), opt_(), keys_(ctx_),
        reference_addkey_(true), result(static_cast<char*>(mr->addr), 0) {
    // room for every key the slot's filter can hold: one pool buffer per builder
    if (bits_per_key > 0) hash_entries_.reserve(static_cast<size_t>(mr->length) * 8u / static_cast<size_t>(bits_per_key) + 64);
  }
  FullFilterBlockBuilder(FilterSlot* mr, int bits_per_key, dlsm_ctx* ctx, BuilderOptions opt = {})
      : slot_{nullptr, 0}, local_mr_(mr), bits_per_key_(bits_per_key),
        num_probes_(dlsm_bloom_full_num_probes(bits_per_key)), ctx_(ctx), opt_(opt), keys_(ctx),
        result(static_cast<char*>(mr->addr), 0) {
    if (opt_.hash_in_addkey) pend_bytes_.resize(kHashBlock * 32);  // a block of 20-byte keys fits
  }
  FullFilterBlockBuilder(const FullFilterBlockBuilder&) = delete;
  FullFilterBlockBuilder& operator=(const FullFilterBlockBuilder&) = delete;

  // full_filter_block.cc:30-33 -- drops the pending keys.
  void RestartBlock(uint64_t /*block_offset*/) {
    hash_entries_.clear();
    clear_keys();
  }
  // full_filter_block.cc:39-49 -- the GPU applies the consecutive-hash dedup.
  // The builder only records the keys (pinned staging) and whether they all
  // have one length (then Finish hands them over as a fixed-stride set: the
  // LDS-tiled key loaders) and whether a key repeats its predecessor (then
  // the line count is counted exactly before bucketing: DLSM_OPT_BUILD_EXACT).
  void AddKey(const Slice& key) {
    if (reference_addkey_) {  // full_filter_block.cc:39-49, unchanged
      const uint32_t hash = BloomHash(key.data(), key.size());
      if (hash_entries_.size() == 0 || hash != hash_entries_.back()) hash_entries_.push_back(hash);
      return;
    }
    if (opt_.hash_in_addkey && key.size() == 20 && pend_fixed20_ && stage_status_ == DLSM_OK) {
      // db_bench's shape: the key joins the pending block (two fixed-size copies)
      char* d = pend_bytes_.data() + pend_size_;
      std::memcpy(d, key.data(), 16);
      std::memcpy(d + 16, key.data() + 16, 4);
      pend_size_ += 20;
      if (++pend_n_ == kHashBlock) hash_pending();
      return;
    }
    add_key_staged(key);  // kept out of line: AddKey itself stays small enough to inline
  }
  // full_filter_block.cc:93-141 -- writes the filter into result.data()'s
  // buffer (the slot, or the buffer given to Move_buffer).
  void Finish() { finish_impl(); }
  void Reset() { result.Reset(static_cast<char*>(local_mr_->addr), 0); }

 private:
  __attribute__((noinline)) void add_key_staged(const Slice& key) {
    if (stage_status_ != DLSM_OK) return;  // staging failed: Finish reports it
    if (opt_.hash_in_addkey) {
      // the key joins a small block of pending keys; every kHashBlock keys
      // the block is hashed at once (independent hash chains overlap) and its
      // hashes staged -- the same values, in the same order, as hashing in
      // every AddKey call
      if (key.size() == 20 && pend_fixed20_) {  // db_bench's shape: two fixed-size copies
        char* d = pend_bytes_.data() + pend_size_;
        std::memcpy(d, key.data(), 16);
        std::memcpy(d + 16, key.data() + 16, 4);
        pend_size_ += 20;
        if (++pend_n_ == kHashBlock) hash_pending();
        return;
      }
      if (pend_fixed20_) {  // a key of another length: the pending ones were all 20 bytes
        for (size_t i = 0; i < pend_n_; i++) pend_len_[i] = 20;
        pend_fixed20_ = false;
      }
      if (pend_size_ + key.size() > pend_bytes_.size())
        pend_bytes_.resize(2 * (pend_size_ + key.size()) + kHashBlock * 32);
      std::memcpy(pend_bytes_.data() + pend_size_, key.data(), key.size());
      pend_size_ += key.size();
      pend_len_[pend_n_++] = static_cast<uint32_t>(key.size());
      if (pend_n_ == kHashBlock) hash_pending();
      return;
    }
    const size_t prev0 = keys_.size() - last_len_;  // the previous key's offset
    if (n_ == 0) {
      key_len_ = key.size();
    } else {
      if (key.size() == last_len_ && memcmp(keys_.data() + prev0, key.data(), last_len_) == 0) dups_++;
      if (uniform_ && key.size() != key_len_) {  // first key of another length: offsets from now on
        uniform_ = false;
        offsets_.resize(n_ + 1);
        for (uint64_t i = 0; i <= n_; i++) offsets_[i] = i * key_len_;
      }
    }
    if (!keys_.append(key.data(), key.size())) {
      stage_status_ = DLSM_E_NOMEM;
      return;
    }
    if (!uniform_) offsets_.push_back(keys_.size());
    last_len_ = key.size();
    n_++;
  }
  void finish_impl() {
    if (reference_addkey_) {
      finish_hash_entries();
      return;
    }
    if (opt_.hash_in_addkey && pend_n_) hash_pending();
    if (stage_status_ != DLSM_OK) {
      // the keys could not all be staged (host memory exhausted): the
      // match-everything filter keeps the table readable and exact in the
      // only sense a Bloom filter must be -- no false negatives
      device_status_ = status_ = stage_status_;
      fell_back_ = false;
      result.Reset(result.data(), host::MatchAllFilter(bits_per_key_, const_cast<char*>(result.data()),
                                                       output_capacity()));
      clear_keys();
      return;
    }
    dlsm_build_job job;
    job.keys.bytes = keys_.data();
    job.keys.n = n_;
    job.keys.suffix_len = 0;
    if (opt_.hash_in_addkey) {  // BloomHash values, already deduplicated
      job.keys.offsets = nullptr;
      job.keys.key_len = 4;
    } else if (uniform_) {
      job.keys.offsets = nullptr;
      job.keys.key_len = static_cast<uint32_t>(key_len_);
    } else {
      job.keys.offsets = offsets_.data();
      job.keys.key_len = 0;
    }
    job.out = reinterpret_cast<uint8_t*>(const_cast<char*>(result.data()));
    job.out_cap = output_capacity();
    uint64_t len = 0;
    // repeated keys lower the line count: have the library count it exactly
    // first (this builder's context belongs to its thread; the caller's
    // setting is restored after the call)
    uint64_t exact = 0;
    const bool own_exact = dups_ && !opt_.batcher && ctx_;
    if (own_exact) {
      dlsm_ctx_get_option(ctx_, DLSM_OPT_BUILD_EXACT, &exact);
      dlsm_ctx_set_option(ctx_, DLSM_OPT_BUILD_EXACT, 1);
    }
    if (opt_.batcher)  // the flag tells the batcher's executor context to count exactly
      status_ = dlsm_batcher_submit(opt_.batcher, &job, bits_per_key_,
                                    (opt_.hash_in_addkey ? DLSM_BATCH_HASHED : 0) | (dups_ ? DLSM_BATCH_EXACT : 0), &len);
    else if (opt_.hash_in_addkey)
      status_ = dlsm_bloom_full_build_hashed(ctx_, &job, 1, bits_per_key_, &len);
    else
      status_ = dlsm_bloom_full_build(ctx_, &job, 1, bits_per_key_, &len);
    if (own_exact) dlsm_ctx_set_option(ctx_, DLSM_OPT_BUILD_EXACT, exact);
    if (!ctx_ && !opt_.batcher) status_ = DLSM_E_DEVICE;
    settle(status_, len, [&](std::vector<uint32_t>& h) { staged_hashes(h); });
    clear_keys();
  }
  // The BloomHash values of the staged keys, in AddKey order (the host
  // fallback's input): the staged hashes themselves with hash_in_addkey,
  // else every key hashed.
  void staged_hashes(std::vector<uint32_t>& h) const {
    if (opt_.hash_in_addkey) {
      h.resize(n_);
      if (n_) std::memcpy(h.data(), keys_.data(), 4 * n_);
      return;
    }
    h.resize(n_);
    const char* b = reinterpret_cast<const char*>(keys_.data());
    for (uint64_t i = 0; i < n_; i++)
      h[i] = uniform_ ? BloomHash(b + i * key_len_, key_len_)
                      : BloomHash(b + offsets_[i], static_cast<size_t>(offsets_[i + 1] - offsets_[i]));
  }
  // The outcome of a Finish whose GPU call returned st (len bytes on
  // success).  On a device-side failure the reference's own loop builds the
  // filter on the host from the hashes get_hashes fills (counted:
  // dlsm_fallback_note); on a slot too small for the filter the
  // match-everything filter goes in its place (status DLSM_E_CAPACITY).  The
  // result is never a 0-byte or partial filter unless the buffer cannot hold
  // even that one (fewer than 69 bytes, or Move_buffer without a size).
  template <class GetHashes>
  void settle(int st, uint64_t len, GetHashes get_hashes) {
    device_status_ = st;
    fell_back_ = false;
    char* out = const_cast<char*>(result.data());
    const size_t cap = output_capacity();
    if (st == DLSM_OK) {
      status_ = DLSM_OK;
      result.Reset(result.data(), len);
      return;
    }
    if (st != DLSM_E_CAPACITY) {
      dlsm_fallback_note(ctx_);
      fell_back_ = true;
      std::vector<uint32_t> h;
      get_hashes(h);
      len = host::FullFilterFromHashes(h.data(), h.size(), bits_per_key_, out, cap, true);
      if (len) {
        status_ = DLSM_OK;
        result.Reset(result.data(), len);
        return;
      }
    }
    status_ = DLSM_E_CAPACITY;
    result.Reset(result.data(), host::MatchAllFilter(bits_per_key_, out, cap));
  }

 public:
  // Output goes to p from now on (full_filter_block.cc:144-146).  Every
  // reference caller moves back into its own slot (local_filter_mr[0]->addr:
  // table_builder_computeside.cc:566, table_builder_bacs.cpp:553,
  // table_builder_bams.cpp:456); a buffer outside the slot must come with its
  // size, or Finish refuses it (DLSM_E_CAPACITY) -- the reference's only
  // check is an assert against the slot's length (full_filter_block.cc:103).
  void Move_buffer(const char* p) { Move_buffer(p, 0); }
  void Move_buffer(const char* p, size_t cap) {
    result.Reset(p, 0);
    moved_cap_ = cap;
  }
  // Bytes Finish may write at result.data(): the rest of the slot when the
  // output lies inside it, else the size given to Move_buffer (0 if none).
  size_t output_capacity() const {
    const char* a = static_cast<const char*>(local_mr_->addr);
    const char* p = result.data();
    if (p >= a && p < a + local_mr_->length) return local_mr_->length - static_cast<size_t>(p - a);
    return moved_cap_;
  }
  int num_probes() const { return num_probes_; }
  // DLSM_OK: `result` is the exact filter of the table's keys (built on the
  // GPU, or by the host loop after a GPU failure: fell_back()).
  // DLSM_E_CAPACITY: the buffer cannot hold it; `result` is the 69-byte
  // match-everything filter (or empty, below 69 bytes).  device_status(): the
  // GPU call's own status.
  int status() const { return status_; }
  int device_status() const { return device_status_; }
  bool fell_back() const { return fell_back_; }

 private:
  // Finish of the reference-signature form: the filter of hash_entries_
  // (CalculateSpace + AddHash + trailer, full_filter_block.cc:93-141) built
  // on the GPU from the 4-byte hashes.
  void finish_hash_entries() {
    dlsm_build_job job;
    job.keys.bytes = reinterpret_cast<const uint8_t*>(hash_entries_.data());
    job.keys.offsets = nullptr;
    job.keys.key_len = 4;
    job.keys.suffix_len = 0;
    job.keys.n = hash_entries_.size();
    job.out = reinterpret_cast<uint8_t*>(const_cast<char*>(result.data()));
    job.out_cap = output_capacity();
    uint64_t len = 0;
    const int st = ctx_ ? dlsm_bloom_full_build_hashed(ctx_, &job, 1, bits_per_key_, &len) : DLSM_E_DEVICE;
    settle(st, len, [&](std::vector<uint32_t>& h) { h.assign(hash_entries_.begin(), hash_entries_.end()); });
    hash_entries_.clear();
  }
  // BloomHash of the pending keys into the staged hashes, dropping a hash
  // equal to its predecessor (full_filter_block.cc:45-48) branch-free: every
  // hash is written, the write position advances only for a kept one.
  void hash_pending() {
    uint8_t* t = keys_.tail(4 * pend_n_ + 64);  // + a 64-byte vector store's overhang
    if (!t) {
      stage_status_ = DLSM_E_NOMEM;
      pend_size_ = pend_n_ = 0;
      pend_fixed20_ = true;
      return;
    }
    uint32_t h[kHashBlock];
    const char* p = pend_bytes_.data();
    size_t i = 0;
    // 20-byte keys 16 at a time (AVX-512) or four at a time (four
    // independent multiply chains); pend_len_ is filled only once the block
    // holds a key of another length
    if (pend_fixed20_) {
      if (HasAvx512())
        for (; i + 16 <= pend_n_; i += 16, p += 320) BloomHash20x16(p, h + i);
      for (; i + 4 <= pend_n_; i += 4, p += 80) BloomHash20x4(p, h + i);
      for (; i < pend_n_; i++, p += 20) h[i] = BloomHash(p, 20);
    } else {
      for (; i + 4 <= pend_n_ && pend_len_[i] == 20 && pend_len_[i + 1] == 20 && pend_len_[i + 2] == 20 &&
             pend_len_[i + 3] == 20;
           i += 4, p += 80)
        BloomHash20x4(p, h + i);
      for (; i < pend_n_; i++) {
        h[i] = BloomHash(p, pend_len_[i]);
        p += pend_len_[i];
      }
    }
    size_t kept = 0;
    uint32_t last = last_hash_;
    const bool first = n_ == 0;
    if (pend_n_ % 16 == 0 && HasAvx512()) {
      kept = DedupStore16(h, pend_n_, last, first, t);
      last = h[pend_n_ - 1];
    } else {
      for (size_t j = 0; j < pend_n_; j++) {
        std::memcpy(t + 4 * kept, &h[j], 4);
        kept += static_cast<size_t>((first && j == 0) | (h[j] != last));
        last = h[j];
      }
    }
    keys_.advance(4 * kept);
    n_ += kept;
    last_hash_ = last;
    pend_size_ = pend_n_ = 0;
    pend_fixed20_ = true;
  }
  void clear_keys() {
    keys_.clear();
    offsets_.clear();
    uniform_ = true;
    key_len_ = last_len_ = 0;
    n_ = dups_ = 0;
    pend_size_ = pend_n_ = 0;
    pend_fixed20_ = true;
    stage_status_ = DLSM_OK;
  }
  FilterSlot slot_;  // the reference-signature form's copy of mr->addr / mr->length
  FilterSlot* local_mr_;
  int bits_per_key_;
  int num_probes_;
  dlsm_ctx* ctx_;
  BuilderOptions opt_;
  PinnedBytes keys_;               // the keys back to back, or their BloomHash values
  uint32_t last_hash_ = 0;         // hash_in_addkey: the last staged hash
  std::vector<uint64_t> offsets_;  // key boundaries, only once lengths differ
  bool uniform_ = true;
  size_t key_len_ = 0, last_len_ = 0;
  // hash_in_addkey: keys pending hashing (bytes back to back + lengths)
  static constexpr size_t kHashBlock = 256;
  std::vector<char> pend_bytes_;  // capacity kept across tables
  uint32_t pend_len_[kHashBlock];
  size_t pend_size_ = 0, pend_n_ = 0;
  bool pend_fixed20_ = true;  // every pending key is 20 bytes
  uint64_t n_ = 0, dups_ = 0;
  size_t moved_cap_ = 0;
  int status_ = DLSM_OK;        // the last Finish's result
  int device_status_ = DLSM_OK;  // the last Finish's GPU call
  bool fell_back_ = false;       // the last Finish's filter came from the host loop
  int stage_status_ = DLSM_OK;  // key staging of the current table
  bool reference_addkey_ = false;
  std::vector<uint32_t, PinnedAllocator<uint32_t>> hash_entries_;  // full_filter_block.h:61

 public:
  Slice result;  // Filter data computed so far
};

// The filter side of a reader (table/full_filter_block.h:25): a Compute-side
// reader owns its filter's FilterChunk slot and frees it in its destructor
// (full_filter_block.cc:285-293).  The reference-signature constructor takes
// the host's own enum as-is (any enum whose Compute is 0).
enum FilterSide { Compute, Memory };

namespace detail {
// Converts to whatever chunk-type enum the manager's
// Deallocate_Local_RDMA_Slot(void*, Chunk_type) takes: FilterChunk = 5
// (util/rdma.h:75).
struct FilterChunkTag {
  template <class E>
  operator E() const {  // NOLINT
    return static_cast<E>(5);
  }
};
// The memory manager a reader holds (std::shared_ptr<RDMA_Manager> in the
// reference), type-erased; Release frees the filter's slot.
struct SlotOwner {
  virtual ~SlotOwner() {}
  virtual void Release(const char* p) = 0;
};
template <class M>
struct ManagerSlotOwner : SlotOwner {
  M mgr;
  explicit ManagerSlotOwner(const M& m) : mgr(m) {}
  void Release(const char* p) override {
    if (mgr) (void)mgr->Deallocate_Local_RDMA_Slot(static_cast<void*>(const_cast<char*>(p)), FilterChunkTag{});
  }
};
}  // namespace detail

// table/full_filter_block.h:71-94.  KeyMayMatch (one key: Table::InternalGet,
// table/table.cc:357) is answered on the host from the filter bytes -- the
// reference's own arithmetic, no device call.  KeysMayMatch (a batch: a
// MultiGet over the version's tables) runs on the GPU; the device copy of the
// filter is made on the first batch, on the calling thread's device, so a
// reader that never batches holds no device memory.
class FullFilterBlockReader {
 public:
  // The reference's signature (full_filter_block.h:76-77):
  // FullFilterBlockReader(const Slice&, std::shared_ptr<RDMA_Manager>, FilterSide).
  // `rdma_mg` is any pointer-like manager with Deallocate_Local_RDMA_Slot(void*,
  // Chunk_type); a Compute-side reader frees the filter's slot through it in
  // its destructor, as the reference does.  Batches use the calling thread's
  // context (dlsm_thread_ctx).  Corrupt metadata -> status() DLSM_E_CORRUPT
  // (the reference exit(1)s) and every probe answers true.
  template <class M, class Side>
  FullFilterBlockReader(const Slice& contents, M rdma_mg, Side side)
      : filter_content(contents), ctx_(nullptr), thread_ctx_(true) {
    if (static_cast<int>(side) == 0) owner_ = new detail::ManagerSlotOwner<M>(rdma_mg);
    parse();
  }
  // The adapter's form: batches run on `ctx` (nullptr: the calling thread's).
  FullFilterBlockReader(const Slice& contents, dlsm_ctx* ctx)
      : filter_content(contents), ctx_(ctx), thread_ctx_(ctx == nullptr) {
    parse();
  }
  ~FullFilterBlockReader() {
    for (dlsm_filterset* f : fs_)
      if (f) dlsm_filterset_destroy(f);
    if (owner_) {
      owner_->Release(filter_content.data());
      delete owner_;
    }
  }
  FullFilterBlockReader(const FullFilterBlockReader&) = delete;
  FullFilterBlockReader& operator=(const FullFilterBlockReader&) = delete;

  // full_filter_block.cc:269-284, on the host.
  bool KeyMayMatch(const Slice& key) const {
    if (meta_.status != DLSM_OK) return true;  // errors are potential matches
    return host::FullHashMayMatch(filter_content.data(), meta_, BloomHash(key.data(), key.size()));
  }
  // Batch form (the GPU's shape): out[i] = 1 if keys[i] may match.  Runs on
  // the GPU; if the device cannot take it (no device, device error, out of
  // memory) the host answers instead (counted: dlsm_fallback_stats), so out
  // is always filled.  Returns DLSM_OK, or DLSM_E_ARG for a null out / keys.
  int KeysMayMatch(const Slice* keys, size_t n, uint8_t* out) {
    if (n == 0) return DLSM_OK;
    if (!keys || !out) return DLSM_E_ARG;
    dlsm_ctx* ctx = thread_ctx_ ? ThreadContext() : ctx_;
    int st = meta_.status == DLSM_OK ? DLSM_OK : meta_.status;
    dlsm_filterset* fs = nullptr;
    if (st == DLSM_OK) st = ctx ? device_set(ctx, &fs) : DLSM_E_DEVICE;
    if (st == DLSM_OK) {
      std::string bytes;
      std::vector<uint64_t> offs(1, 0);
      offs.reserve(n + 1);
      for (size_t i = 0; i < n; i++) {
        bytes.append(keys[i].data(), keys[i].size());
        offs.push_back(bytes.size());
      }
      if (bytes.empty()) bytes.push_back('\0');
      dlsm_keyset ks{reinterpret_cast<const uint8_t*>(bytes.data()), offs.data(), 0, 0, n};
      st = dlsm_bloom_full_probe(ctx, fs, &ks, out);
    }
    last_device_status_ = st;
    if (st != DLSM_OK) {
      if (meta_.status == DLSM_OK) dlsm_fallback_note(ctx);  // a corrupt filter is not a device failure
      for (size_t i = 0; i < n; i++) out[i] = KeyMayMatch(keys[i]) ? 1 : 0;
    }
    return DLSM_OK;
  }
  int status() const { return meta_.status; }
  int num_probes() const { return meta_.k; }
  uint32_t num_lines() const { return meta_.num_lines; }
  // The last batch's GPU status (DLSM_OK when the device answered it).
  int last_device_status() const { return last_device_status_; }
  // Whether a device copy of the filter exists (made by the first batch).
  bool device_resident() const {
    for (dlsm_filterset* f : fs_)
      if (f) return true;
    return false;
  }

  Slice filter_content;

 private:
  void parse() { meta_ = host::ParseFull(filter_content.data(), filter_content.size()); }
  // The filter's device copy on ctx's device, made on first use.  Readers are
  // shared by reader threads (table_cache.cc:292-299): one copy per device.
  int device_set(dlsm_ctx* ctx, dlsm_filterset** out) {
    const int dev = dlsm_ctx_device(ctx);
    if (dev < 0) return DLSM_E_DEVICE;
    std::lock_guard<std::mutex> lk(mu_);
    if (fs_.size() <= static_cast<size_t>(dev)) fs_.resize(static_cast<size_t>(dev) + 1, nullptr);
    if (!fs_[dev]) {
      const uint8_t* f = reinterpret_cast<const uint8_t*>(filter_content.data());
      const uint64_t len = filter_content.size();
      const int st = dlsm_filterset_create(ctx, &f, &len, 1, 0, &fs_[dev]);
      if (st != DLSM_OK) {
        fs_[dev] = nullptr;
        return st;
      }
    }
    *out = fs_[dev];
    return DLSM_OK;
  }
  dlsm_ctx* ctx_;
  bool thread_ctx_;
  detail::SlotOwner* owner_ = nullptr;
  host::FullFilterMeta meta_;
  std::mutex mu_;
  std::vector<dlsm_filterset*> fs_;  // by device
  int last_device_status_ = DLSM_OK;
};

// The legacy-format policy (util/bloom.cc:14-91) as a FilterPolicy.
// Name() keeps the reference's format identity string.  suffix_len() = 8
// makes it hash ExtractUserKey(key) of internal keys (the form
// InternalFilterPolicy wraps it in).  CreateFilter runs on the GPU (ctx, or
// the calling thread's context when ctx is nullptr), falling back to the
// reference's loop on the host if the device cannot take it (counted);
// KeyMayMatch is one key, answered on the host.
class BloomFilterPolicy : public FilterPolicy {
 public:
  // util/bloom.cc:16 -- the reference's signature; builds on the calling
  // thread's context.
  explicit BloomFilterPolicy(int bits_per_key) : BloomFilterPolicy(bits_per_key, nullptr) {}
  BloomFilterPolicy(int bits_per_key, dlsm_ctx* ctx, uint32_t suffix_len = 0)
      : bits_per_key_(bits_per_key), ctx_(ctx), suffix_len_(suffix_len) {}
  const char* Name() const override { return "TimberSaw.BuiltinBloomFilter2"; }

  // Append a filter summarising keys[0, n) to *dst (util/bloom.cc:25-55).
  void CreateFilter(const Slice* keys, int n, Slice* dst) const override {
    const int nn = n < 0 ? 0 : n;
    std::string bytes;
    std::vector<uint64_t> offs(1, 0);
    offs.reserve(static_cast<size_t>(nn) + 1);
    for (int i = 0; i < nn; i++) {
      bytes.append(keys[i].data(), keys[i].size());
      offs.push_back(bytes.size());
    }
    if (bytes.empty()) bytes.push_back('\0');
    uint64_t need = 0;
    dlsm_bloom_legacy_size(static_cast<uint64_t>(nn), bits_per_key_, &need);
    char* out = const_cast<char*>(dst->data()) + dst->size();
    dlsm_build_job job;
    job.keys = dlsm_keyset{reinterpret_cast<const uint8_t*>(bytes.data()), offs.data(), 0, suffix_len_,
                           static_cast<uint64_t>(nn)};
    job.out = reinterpret_cast<uint8_t*>(out);
    job.out_cap = need;
    uint64_t len = 0;
    dlsm_ctx* ctx = ctx_ ? ctx_ : ThreadContext();
    last_status_ = ctx ? dlsm_bloom_legacy_build(ctx, &job, 1, bits_per_key_, &len) : DLSM_E_DEVICE;
    if (last_status_ != DLSM_OK) {
      dlsm_fallback_note(ctx);
      len = host::LegacyCreateFilter(keys, nn, bits_per_key_, suffix_len_, out);
    }
    dst->Reset(dst->data(), dst->size() + len);
  }
  // util/bloom.cc:57-81, on the host.
  bool KeyMayMatch(const Slice& key, const Slice& filter) const override {
    const size_t len = key.size() >= suffix_len_ ? key.size() - suffix_len_ : 0;
    return host::LegacyKeyMayMatch(key.data(), len, filter.data(), filter.size());
  }
  int bits_per_key() const { return bits_per_key_; }
  dlsm_ctx* ctx() const { return ctx_; }
  uint32_t suffix_len() const { return suffix_len_; }
  // The last CreateFilter's GPU status (the filter is complete either way).
  int status() const { return last_status_; }

 private:
  int bits_per_key_;
  dlsm_ctx* ctx_;
  uint32_t suffix_len_;
  mutable int last_status_ = DLSM_OK;
};

// util/bloom.cc:89-91 and include/TimberSaw/filter_policy.h:71 -- the
// reference's signature (db_bench: NewBloomFilterPolicy(FLAGS_bloom_bits),
// benchmarks/db_bench.cc:638); builds on the calling thread's context.  The
// caller deletes the result (after every DB using it is closed).
inline const FilterPolicy* NewBloomFilterPolicy(int bits_per_key) { return new BloomFilterPolicy(bits_per_key); }
// The same on a given context.
inline const FilterPolicy* NewBloomFilterPolicy(int bits_per_key, dlsm_ctx* ctx) {
  return new BloomFilterPolicy(bits_per_key, ctx);
}

// db/dbformat.h:399-408, db/dbformat.cc:93-109: converts internal keys to
// user keys for the wrapped policy.
//  * wrapping this header's BloomFilterPolicy: the internal keys go to the
//    GPU as they are, with suffix_len = 8 -- the kernels hash
//    ExtractUserKey(key), no host-side stripping pass;
//  * wrapping any other FilterPolicy: keys[] is rewritten to the user keys
//    and handed on, exactly as the reference does ("the code in table.cc
//    does not mind us adjusting keys[]").
// The reference rewrites keys[] in both cases; so does this class, so a
// caller sees the same keys[] afterwards.
class InternalFilterPolicy : public FilterPolicy {
 public:
  explicit InternalFilterPolicy(const FilterPolicy* p) : user_policy_(p) {}
  explicit InternalFilterPolicy(const BloomFilterPolicy* p)
      : user_policy_(p), gpu_(p->bits_per_key(), p->ctx(), DLSM_INTERNAL_KEY_TRAILER) {
    gpu_ok_ = true;
  }
  const char* Name() const override { return user_policy_->Name(); }
  void CreateFilter(const Slice* keys, int n, Slice* dst) const override {
    if (gpu_ok_) gpu_.CreateFilter(keys, n, dst);
    Slice* mkey = const_cast<Slice*>(keys);
    for (int i = 0; i < n; i++) mkey[i] = ExtractUserKey(keys[i]);
    if (!gpu_ok_) user_policy_->CreateFilter(keys, n, dst);
  }
  bool KeyMayMatch(const Slice& key, const Slice& f) const override {
    if (gpu_ok_) return gpu_.KeyMayMatch(key, f);
    return user_policy_->KeyMayMatch(ExtractUserKey(key), f);
  }
  int status() const { return gpu_ok_ ? gpu_.status() : DLSM_OK; }

 private:
  const FilterPolicy* const user_policy_;
  BloomFilterPolicy gpu_{0, nullptr};
  bool gpu_ok_ = false;
};

// table/filter_block.cc:14-113 with the legacy Bloom policy.  StartBlock /
// AddKey only record the call sequence; Finish builds every filter of the
// block on the GPU and writes the block (filters, offsets, array offset,
// kFilterBaseLg) into the slot.
class FilterBlockBuilder {
 public:
  FilterBlockBuilder(FilterSlot* mr, int bits_per_key, dlsm_ctx* ctx)
      : result(static_cast<char*>(mr->addr), 0), local_mr_(mr), bits_per_key_(bits_per_key), ctx_(ctx) {
    offsets_.push_back(0);
  }
  FilterBlockBuilder(const FilterBlockBuilder&) = delete;
  FilterBlockBuilder& operator=(const FilterBlockBuilder&) = delete;

  void StartBlock(uint64_t block_offset) {
    block_key_end_.push_back(offsets_.size() - 1);
    block_end_offset_.push_back(block_offset);
  }
  void AddKey(const Slice& key) {
    keys_.append(key.data(), key.size());
    offsets_.push_back(keys_.size());
  }
  Slice Finish() {
    dlsm_keyset ks{reinterpret_cast<const uint8_t*>(keys_.data()), offsets_.data(), 0, 0,
                   offsets_.size() - 1};
    uint64_t len = 0;
    dlsm_ctx* ctx = ctx_ ? ctx_ : ThreadContext();
    status_ = ctx ? dlsm_filter_block_build(ctx, &ks, block_key_end_.data(), block_end_offset_.data(),
                                            static_cast<int>(block_key_end_.size()), bits_per_key_,
                                            reinterpret_cast<uint8_t*>(local_mr_->addr), local_mr_->length, &len)
                  : DLSM_E_DEVICE;
    if (status_ != DLSM_OK && status_ != DLSM_E_CAPACITY) {
      dlsm_fallback_note(ctx);
      len = host_finish();
      status_ = len ? DLSM_OK : DLSM_E_CAPACITY;
    }
    result.Reset(static_cast<char*>(local_mr_->addr), status_ == DLSM_OK ? len : 0);
    return result;
  }
  void Reset() { result.Reset(static_cast<char*>(local_mr_->addr), 0); }
  int status() const { return status_; }

  Slice result;

 private:
  // filter_block.cc:32-113 on the host (the GPU call failed): replays the
  // recorded StartBlock / AddKey sequence -- a filter per 2 KiB of block
  // offsets (GenerateFilter at each StartBlock that crosses into a later
  // 2 KiB range, and at Finish for keys still pending), then the Fixed32
  // offsets, the array offset and kFilterBaseLg.  Returns the block's length,
  // 0 if the slot is too small.
  uint64_t host_finish() {
    const size_t n_keys = offsets_.size() - 1;
    uint64_t need = 5;
    size_t done = 0;  // keys already in a filter
    std::vector<uint32_t> foffs;
    std::vector<Slice> tmp;
    char* out = static_cast<char*>(local_mr_->addr);
    const size_t cap = local_mr_->length;
    auto generate = [&](size_t upto) -> bool {
      foffs.push_back(static_cast<uint32_t>(need - 5));
      if (upto == done) return true;
      uint64_t sz = 0;
      dlsm_bloom_legacy_size(upto - done, bits_per_key_, &sz);
      if (need + sz + 4 * (foffs.size() + 1) > cap) return false;
      tmp.clear();
      for (size_t i = done; i < upto; i++)
        tmp.emplace_back(keys_.data() + offsets_[i], static_cast<size_t>(offsets_[i + 1] - offsets_[i]));
      host::LegacyCreateFilter(tmp.data(), static_cast<int>(tmp.size()), bits_per_key_, 0, out + need - 5);
      need += sz;
      done = upto;
      return true;
    };
    for (size_t b = 0; b < block_key_end_.size(); b++) {
      const uint64_t index = block_end_offset_[b] >> 11;  // kFilterBaseLg
      while (index > foffs.size())
        if (!generate(static_cast<size_t>(block_key_end_[b]))) return 0;
    }
    if (done < n_keys && !generate(n_keys)) return 0;
    const uint64_t array_offset = need - 5;
    if (array_offset + 4 * foffs.size() + 5 > cap) return 0;
    char* p = out + array_offset;
    for (uint32_t f : foffs) {
      host::PutFixed32(p, f);
      p += 4;
    }
    host::PutFixed32(p, static_cast<uint32_t>(array_offset));
    p[4] = 11;
    return array_offset + 4 * foffs.size() + 5;
  }
  FilterSlot* local_mr_;
  int bits_per_key_;
  dlsm_ctx* ctx_;
  std::string keys_;
  std::vector<uint64_t> offsets_;
  std::vector<uint64_t> block_key_end_, block_end_offset_;
  int status_ = DLSM_OK;
};

// table/filter_block.h:70-85.  KeyMayMatch (one key) on the host from the
// block's bytes; KeysMayMatch (a batch) on the GPU (ctx, or the calling
// thread's context when ctx is nullptr).
class FilterBlockReader {
 public:
  FilterBlockReader(const Slice& contents, dlsm_ctx* ctx) : contents_(contents), ctx_(ctx) {}
  // filter_block.cc:127-142, on the host.
  bool KeyMayMatch(uint64_t block_offset, const Slice& key) const {
    return host::FilterBlockKeyMayMatch(contents_.data(), contents_.size(), block_offset, key.data(), key.size());
  }
  int KeysMayMatch(const uint64_t* block_offsets, const Slice* keys, size_t n, uint8_t* out) {
    dlsm_ctx* ctx = ctx_ ? ctx_ : ThreadContext();
    const int st = ctx ? device_batch(ctx, block_offsets, keys, n, out) : DLSM_E_DEVICE;
    if (st != DLSM_OK && n && keys && out && block_offsets) {  // the host answers instead (counted)
      dlsm_fallback_note(ctx);
      for (size_t i = 0; i < n; i++) out[i] = KeyMayMatch(block_offsets[i], keys[i]) ? 1 : 0;
      return DLSM_OK;
    }
    return st;
  }

 private:
  int device_batch(dlsm_ctx* ctx, const uint64_t* block_offsets, const Slice* keys, size_t n, uint8_t* out) {
    std::string bytes;
    std::vector<uint64_t> offs(1, 0);
    for (size_t i = 0; i < n; i++) {
      bytes.append(keys[i].data(), keys[i].size());
      offs.push_back(bytes.size());
    }
    if (bytes.empty()) bytes.push_back('\0');
    dlsm_keyset ks{reinterpret_cast<const uint8_t*>(bytes.data()), offs.data(), 0, 0, n};
    return dlsm_filter_block_probe(ctx, reinterpret_cast<const uint8_t*>(contents_.data()),
                                   contents_.size(), &ks, block_offsets, out);
  }
  Slice contents_;
  dlsm_ctx* ctx_;
};

}  // namespace dlsm_adapter
