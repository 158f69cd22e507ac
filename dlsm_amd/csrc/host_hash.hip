// dlsm_amd/csrc/host_hash.hip -- BloomHash of a batch of host keys on the
// host's cores (host code only; no device work).
//
// The reference hashes on the host: FullFilterBlockBuilder::AddKey
// (table/full_filter_block.cc:45) and FullFilterBlockReader::KeyMayMatch
// (:271) call BloomHash (include/TimberSaw/filter_policy.h:26-28,
// util/hash.cc:22-62) per key.  A caller whose keys live in host memory
// (memtable / compaction iterators, Get() callers) can hash them here and
// hand the GPU 4 bytes per key (dlsm_bloom_full_build_hashed*,
// dlsm_bloom_full_probe_hashed_dev) instead of the key bytes: a quarter of
// the PCIe traffic for 20-byte keys.  Thirty-two 20-byte keys at a time with
// AVX-512 when the CPU has it, on a process-wide pool of host threads.
#include <hip/hip_runtime.h>  // bloom_math.h's host/device qualifiers

#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "../../include/dlsm_bloom.h"
#include "bloom_math.h"

namespace {

using dlsm::bloom_hash_host;
using dlsm::hash_init;
using dlsm::hash_word;
using dlsm::kBloomSeed;
using dlsm::kHashM;

#if defined(__x86_64__)
// One 16-key group's gather indices and masks, per round j (constants).
struct Group16 {
  __m512i d[5];
  __mmask16 ge32[5], ge64[5];
};
__attribute__((target("avx512f"))) inline Group16 group16() {
  Group16 g;
  const __m512i q5 = _mm512_mullo_epi32(_mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15),
                                        _mm512_set1_epi32(5));
  for (int j = 0; j < 5; j++) {
    g.d[j] = _mm512_add_epi32(q5, _mm512_set1_epi32(j));
    g.ge32[j] = _mm512_cmpge_epu32_mask(g.d[j], _mm512_set1_epi32(32));
    g.ge64[j] = _mm512_cmpge_epu32_mask(g.d[j], _mm512_set1_epi32(64));
  }
  return g;
}
// Dword j of the sixteen 20-byte keys held in v0..v4 (key q's dword j is
// dword 5q + j of the 320 bytes): two-source permutes + blends.
__attribute__((target("avx512f"))) inline __m512i word16(const Group16& g, int j, __m512i v0, __m512i v1,
                                                         __m512i v2, __m512i v3, __m512i v4) {
  const __m512i lo = _mm512_permutex2var_epi32(v0, g.d[j], v1);
  const __m512i mid = _mm512_permutex2var_epi32(v2, g.d[j], v3);
  const __m512i hi = _mm512_permutexvar_epi32(g.d[j], v4);
  return _mm512_mask_blend_epi32(g.ge64[j], _mm512_mask_blend_epi32(g.ge32[j], lo, mid), hi);
}
// Keys [0, n) of the fixed 20-byte batch at p (n a multiple of 32): util/hash.cc's
// five rounds on two groups of sixteen keys at once -- two independent
// multiply chains per iteration (the round's multiply latency is the
// critical path) -- with the key stream prefetched 2 KiB ahead.
__attribute__((target("avx512f"))) void hash20_avx512(const uint8_t* p, uint64_t n, uint32_t* out) {
  const Group16 g = group16();
  const __m512i m = _mm512_set1_epi32(static_cast<int>(kHashM));
  const __m512i h0 = _mm512_set1_epi32(static_cast<int>(hash_init(20, kBloomSeed)));
  for (uint64_t i = 0; i < n; i += 32, p += 640, out += 32) {
    for (int c = 0; c < 640; c += 64) _mm_prefetch(reinterpret_cast<const char*>(p + 2048 + c), _MM_HINT_T0);
    const __m512i a0 = _mm512_loadu_si512(p), a1 = _mm512_loadu_si512(p + 64), a2 = _mm512_loadu_si512(p + 128),
                  a3 = _mm512_loadu_si512(p + 192), a4 = _mm512_loadu_si512(p + 256);
    const __m512i b0 = _mm512_loadu_si512(p + 320), b1 = _mm512_loadu_si512(p + 384),
                  b2 = _mm512_loadu_si512(p + 448), b3 = _mm512_loadu_si512(p + 512),
                  b4 = _mm512_loadu_si512(p + 576);
    __m512i ha = h0, hb = h0;
    for (int j = 0; j < 5; j++) {
      ha = _mm512_mullo_epi32(_mm512_add_epi32(ha, word16(g, j, a0, a1, a2, a3, a4)), m);
      hb = _mm512_mullo_epi32(_mm512_add_epi32(hb, word16(g, j, b0, b1, b2, b3, b4)), m);
      ha = _mm512_xor_si512(ha, _mm512_srli_epi32(ha, 16));
      hb = _mm512_xor_si512(hb, _mm512_srli_epi32(hb, 16));
    }
    _mm512_storeu_si512(out, ha);
    _mm512_storeu_si512(out + 16, hb);
  }
}
bool has_avx512() {
  static const bool has = __builtin_cpu_supports("avx512f");
  return has;
}
#else
bool has_avx512() { return false; }
void hash20_avx512(const uint8_t*, uint64_t, uint32_t*) {}
#endif

uint32_t hash20(const uint8_t* p) {
  uint32_t w[5];
  std::memcpy(w, p, 20);  // little-endian host, like DecodeFixed32
  uint32_t h = hash_init(20, kBloomSeed);
  for (int j = 0; j < 5; j++) h = hash_word(h, w[j]);
  return h;
}

// keys [lo, hi) of ks
void hash_range(const dlsm_keyset& ks, uint64_t lo, uint64_t hi, uint32_t* out) {
  const uint32_t sfx = ks.suffix_len;
  if (!ks.offsets && ks.key_len == 20 + sfx) {
    const uint64_t stride = ks.key_len;
    uint64_t i = lo;
    if (sfx == 0 && has_avx512() && hi - lo >= 32) {
      const uint64_t n32 = (hi - lo) & ~uint64_t(31);
      hash20_avx512(ks.bytes + lo * 20, n32, out + lo);
      i = lo + n32;
    }
    for (; i < hi; i++) out[i] = hash20(ks.bytes + i * stride);
    return;
  }
  for (uint64_t i = lo; i < hi; i++) {
    uint64_t s, l;
    if (ks.offsets) {
      s = ks.offsets[i];
      l = ks.offsets[i + 1] - s;
    } else {
      s = i * ks.key_len;
      l = ks.key_len;
    }
    l = l > sfx ? l - sfx : 0;  // ExtractUserKey (db/dbformat.h:374-377)
    out[i] = bloom_hash_host(ks.bytes + s, l);
  }
}

// Host cores this process may use: its CPU affinity set, capped by a cgroup
// (v2) CPU quota when one is set -- on a shared GPU box the machine's CPU
// count (hardware_concurrency) is many times the process's share.
int usable_cores() {
  int n = static_cast<int>(std::max(1u, std::thread::hardware_concurrency()));
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = std::max(1, CPU_COUNT(&set));
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long period = 0;
    if (std::fscanf(f, "%31s %lld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0) {
      const long long quota = std::atoll(q);
      if (quota > 0) n = std::min<int>(n, static_cast<int>(std::max(1LL, (quota + period - 1) / period)));
    }
    std::fclose(f);
  }
  return std::min(n, 64);
}

// The NUMA node holding the bytes [p, p + n): the node of three sampled pages
// when they agree, else -1 (move_pages with no target nodes only reports).
int numa_node_of(const void* p, uint64_t n) {
  if (!p || n == 0) return -1;
  const long page = sysconf(_SC_PAGESIZE);
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  void* pages[3];
  for (int i = 0; i < 3; i++)
    pages[i] = reinterpret_cast<void*>((a + (n - 1) * static_cast<uint64_t>(i) / 2) & ~static_cast<uintptr_t>(page - 1));
  int status[3] = {-1, -1, -1};
  if (syscall(SYS_move_pages, 0, 3L, pages, nullptr, status, 0) != 0) return -1;
  return status[0] >= 0 && status[0] == status[1] && status[1] == status[2] ? status[0] : -1;
}

// CPUs of NUMA node `node` that this process may use (empty if none / unknown).
cpu_set_t node_cpus(int node, const cpu_set_t& allowed) {
  cpu_set_t set;
  CPU_ZERO(&set);
  char path[96];
  std::snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = std::fopen(path, "r");
  if (!f) return set;
  char buf[4096] = {0};
  const size_t len = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[len] = 0;
  for (char* s = buf; *s;) {  // "0-63,128-191"
    char* e = nullptr;
    const long lo = std::strtol(s, &e, 10);
    if (e == s) break;
    long hi = lo;
    if (*e == '-') hi = std::strtol(e + 1, &e, 10);
    for (long c = lo; c <= hi && c < CPU_SETSIZE; c++)
      if (CPU_ISSET(c, &allowed)) CPU_SET(c, &set);
    s = (*e == ',') ? e + 1 : e;
    if (*s == '\n') break;
  }
  return set;
}

// A process-wide fork-join pool: run(parts, f) calls f(0..parts-1) on the
// pool's threads and the caller, returning when all are done.  One run at a
// time (callers serialise on run_m).  run(..., node): the pool's threads
// move onto the CPUs of NUMA node `node` first (the node holding the keys:
// hashing reads them from local DRAM instead of across the socket link; the
// caller's own thread is left where it is), node < 0 leaves them as they are.
class Pool {
 public:
  static Pool& get() {
    static Pool p;
    return p;
  }
  int size() const { return static_cast<int>(th_.size()) + 1; }
  void run(int parts, const std::function<void(int)>& f, int node = -1) {
    std::lock_guard<std::mutex> one(run_m_);
    {
      std::lock_guard<std::mutex> lk(m_);
      if (node != node_) {
        node_ = node;
        place_gen_++;
        CPU_ZERO(&place_);
        if (node >= 0) place_ = node_cpus(node, allowed_);
        if (CPU_COUNT(&place_) == 0) place_ = allowed_;  // unknown node: anywhere allowed
      }
      f_ = &f;
      parts_ = parts;
      next_.store(0);
      active_ = static_cast<int>(th_.size());
      gen_++;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return active_ == 0; });
    f_ = nullptr;
  }

 private:
  Pool() {
    if (sched_getaffinity(0, sizeof(allowed_), &allowed_) != 0) {
      CPU_ZERO(&allowed_);
      for (int c = 0; c < CPU_SETSIZE; c++) CPU_SET(c, &allowed_);
    }
    place_ = allowed_;
    const int n = usable_cores() - 1;
    for (int t = 0; t < n; t++) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void work() {
    for (int i; (i = next_.fetch_add(1)) < parts_;) (*f_)(i);
  }
  void loop() {
    uint64_t seen = 0, placed = 0;
    for (;;) {
      cpu_set_t want;
      bool move = false;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        if (placed != place_gen_) {
          placed = place_gen_;
          want = place_;
          move = true;
        }
      }
      if (move) (void)sched_setaffinity(0, sizeof(want), &want);  // this thread only
      work();
      std::lock_guard<std::mutex> lk(m_);
      if (--active_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_, run_m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* f_ = nullptr;
  std::atomic<int> next_{0};
  int parts_ = 0, active_ = 0;
  uint64_t gen_ = 0, place_gen_ = 0;
  bool stop_ = false;
  int node_ = -1;
  cpu_set_t allowed_, place_;
};

}  // namespace

extern "C" int dlsm_bloom_hash_batch(const dlsm_keyset* keys, uint32_t* out, int threads) {
  if (!keys || threads < 0) return DLSM_E_ARG;
  const dlsm_keyset ks = *keys;
  if (ks.n == 0) return DLSM_OK;
  if (!out || !ks.bytes || ks.suffix_len > 255 || (!ks.offsets && ks.key_len < ks.suffix_len)) return DLSM_E_ARG;
  constexpr uint64_t kPart = 1u << 14;  // keys per task (a multiple of 32)
  const uint64_t parts = (ks.n + kPart - 1) / kPart;
  Pool& pool = Pool::get();
  const int width = threads == 0 ? pool.size() : std::min(threads, pool.size());
  if (width <= 1 || parts == 1) {
    hash_range(ks, 0, ks.n, out);
    return DLSM_OK;
  }
  // the pool's threads go to the NUMA node that holds the keys ($DLSM_HASH_NUMA=0: left anywhere)
  static const bool numa = [] {
    const char* e = getenv("DLSM_HASH_NUMA");
    return !(e && atoi(e) == 0);
  }();
  const uint64_t key_bytes = ks.offsets ? ks.offsets[ks.n] : ks.n * static_cast<uint64_t>(ks.key_len);
  const int node = numa ? numa_node_of(ks.bytes, key_bytes) : -1;
  // `width` interleaved lanes of tasks: lane t takes parts t, t + width, ...
  pool.run(width, [&](int t) {
    for (uint64_t p = static_cast<uint64_t>(t); p < parts; p += static_cast<uint64_t>(width))
      hash_range(ks, p * kPart, std::min(ks.n, (p + 1) * kPart), out);
  }, node);
  return DLSM_OK;
}

extern "C" int dlsm_host_read_bytes(const void* p, uint64_t n, int threads, uint64_t* fold) {
  if (!fold || threads < 0 || (n && !p) || (n & 7u)) return DLSM_E_ARG;
  *fold = 0;
  if (n == 0) return DLSM_OK;
  static const bool numa = [] {
    const char* e = getenv("DLSM_HASH_NUMA");
    return !(e && atoi(e) == 0);
  }();
  const uint64_t* w = static_cast<const uint64_t*>(p);
  const uint64_t words = n / 8;
  constexpr uint64_t kPart = 1u << 16;  // words per task (512 KiB)
  const uint64_t parts = (words + kPart - 1) / kPart;
  Pool& pool = Pool::get();
  const int width = threads == 0 ? pool.size() : std::min(threads, pool.size());
  std::vector<uint64_t> acc(static_cast<size_t>(width) * 8, 0);  // a cache line per lane
  auto range = [&](uint64_t lo, uint64_t hi, uint64_t& a) {
    uint64_t x0 = 0, x1 = 0, x2 = 0, x3 = 0;  // four chains: the loop streams, it does not wait on one xor
    uint64_t i = lo;
    for (; i + 4 <= hi; i += 4) {
      x0 ^= w[i];
      x1 ^= w[i + 1];
      x2 ^= w[i + 2];
      x3 ^= w[i + 3];
    }
    for (; i < hi; i++) x0 ^= w[i];
    a ^= x0 ^ x1 ^ x2 ^ x3;
  };
  if (width <= 1 || parts == 1) {
    range(0, words, acc[0]);
  } else {
    pool.run(width, [&](int t) {
      for (uint64_t q = static_cast<uint64_t>(t); q < parts; q += static_cast<uint64_t>(width))
        range(q * kPart, std::min(words, (q + 1) * kPart), acc[static_cast<size_t>(t) * 8]);
    }, numa ? numa_node_of(p, n) : -1);
  }
  for (int t = 0; t < width; t++) *fold ^= acc[static_cast<size_t>(t) * 8];
  return DLSM_OK;
}
