// CPU test of the adapter's host-side AddKey hashing (hash_in_addkey): the
// hashes FullFilterBlockBuilder hands to dlsm_bloom_full_build_hashed must be
// BloomHash of every key with a hash equal to its predecessor dropped
// (full_filter_block.cc:39-49) -- through the 20-byte fast path, the AVX-512
// block hashing and compress-store dedup, the four-chain path and the scalar
// path, across block boundaries and key-length changes.  The few C ABI entry
// points the builder calls are stubbed here (host memory, no GPU), so this
// runs in the CPU suite; tests/cpp/adapter_test.cc checks the same builder's
// filters on the GPU.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "dlsm_bloom_adapter.hpp"

static std::vector<uint32_t> g_staged;  // what the last Finish handed over

extern "C" {
int dlsm_bloom_full_num_probes(int) { return 6; }
int dlsm_ctx_host_buffer_claim(dlsm_ctx*, const void*) { return DLSM_E_BUSY; }
int dlsm_ctx_host_buffer_release(dlsm_ctx*, const void*) { return DLSM_OK; }
int dlsm_ctx_host_buffer(dlsm_ctx*, uint64_t, uint64_t, void**, uint64_t*) { return DLSM_E_ARG; }
int dlsm_host_pool_acquire(uint64_t min_bytes, void** out, uint64_t* cap) {
  const uint64_t c = (min_bytes + 4095) & ~uint64_t(4095);
  *out = std::aligned_alloc(4096, c);
  std::memset(*out, 0xA5, c);  // garbage past the staged hashes must never be handed over
  *cap = c;
  return *out ? DLSM_OK : DLSM_E_NOMEM;
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
int dlsm_bloom_full_build(dlsm_ctx*, const dlsm_build_job*, int, int, uint64_t*) { return DLSM_E_ARG; }
int dlsm_bloom_full_build_hashed(dlsm_ctx*, const dlsm_build_job* j, int n_jobs, int, uint64_t* len) {
  if (n_jobs != 1 || j->keys.key_len != 4 || j->keys.offsets) return DLSM_E_ARG;
  const uint32_t* h = reinterpret_cast<const uint32_t*>(j->keys.bytes);
  g_staged.assign(h, h + j->keys.n);
  *len = 5;
  return DLSM_OK;
}
int dlsm_batcher_full_build(dlsm_batcher*, const dlsm_build_job*, int, uint64_t*) { return DLSM_E_ARG; }
int dlsm_batcher_full_build_hashed(dlsm_batcher*, const dlsm_build_job*, int, uint64_t*) { return DLSM_E_ARG; }
int dlsm_batcher_submit(dlsm_batcher*, const dlsm_build_job*, int, int, uint64_t*) { return DLSM_E_ARG; }
int dlsm_bloom_full_size(uint64_t n, int bpk, uint32_t* L, uint64_t* nbytes) {  // the host fallback's sizing
  uint32_t lines = n ? (static_cast<uint32_t>(n * bpk) + 511) / 512 : 0;
  if (lines && lines % 2 == 0) lines++;
  if (L) *L = lines;
  if (nbytes) *nbytes = uint64_t(lines) * 64 + 5;
  return DLSM_OK;
}
void dlsm_fallback_note(dlsm_ctx*) {}
static int g_thread_ctx_token;
int dlsm_thread_ctx(dlsm_ctx** out) {
  *out = reinterpret_cast<dlsm_ctx*>(&g_thread_ctx_token);  // only passed to the stubs
  return DLSM_OK;
}
}

// an ibv_mr-shaped region (addr + length among other fields)
struct MrShaped {
  void* context;
  void* pd;
  void* addr;
  size_t length;
  uint32_t handle, lkey, rkey;
};

#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      return 1;                                               \
    }                                                         \
  } while (0)

static uint32_t lcg(uint32_t& x) { return x = x * 1664525u + 1013904223u; }

// Both forms hand the same hashes over: hash_in_addkey (block hashing) and
// the reference-signature builder (the reference's per-key AddKey into
// hash_entries_).
static int run(dlsm_adapter::FullFilterBlockBuilder& b, int& cases) {
  for (int shape = 0; shape < 6; shape++) {
    for (int n : {0, 1, 15, 16, 17, 255, 256, 257, 4099, 70001}) {
      uint32_t x = 12345u + static_cast<uint32_t>(shape * 1000 + n);
      std::vector<std::string> keys;
      for (int i = 0; i < n; i++) {
        std::string k;
        const bool k20 = shape == 0 || shape == 3 || (shape == 2 && (i / 250) % 2 == 0) ||
                         (shape == 4 && i % 97 != 5) || (shape == 5 && i == 0);
        if (k20) {
          char buf[21];
          std::snprintf(buf, sizeof(buf), "%020u", shape == 3 ? 7u : lcg(x) % 50000u);  // 3: one key only
          k.assign(buf, 20);
        } else {
          const int len = static_cast<int>(lcg(x) >> 27);  // 0..31 bytes, >= 0x80 included
          for (int q = 0; q < len; q++) k.push_back(static_cast<char>(lcg(x) >> 24));
        }
        keys.push_back(k);
        if (lcg(x) % 9 == 0) keys.push_back(k);  // consecutive duplicates
      }
      b.RestartBlock(0);
      for (const auto& k : keys) b.AddKey(dlsm_adapter::Slice(k));
      g_staged.clear();
      b.Finish();
      CHECK(b.status() == DLSM_OK);
      std::vector<uint32_t> want;
      for (size_t i = 0; i < keys.size(); i++) {
        const uint32_t h = dlsm_adapter::BloomHash(keys[i].data(), keys[i].size());
        if (want.empty() || h != want.back()) want.push_back(h);
      }
      if (want.empty()) {
        CHECK(g_staged.empty());
      } else {
        CHECK(g_staged.size() == want.size());
        CHECK(std::memcmp(g_staged.data(), want.data(), 4 * want.size()) == 0);
      }
      cases++;
    }
  }
  return 0;
}

int main() {
  std::vector<char> slot(1 << 16);
  dlsm_adapter::FilterSlot mr{slot.data(), slot.size()};
  dlsm_adapter::BuilderOptions opt;
  opt.hash_in_addkey = true;
  dlsm_ctx* fake_ctx = reinterpret_cast<dlsm_ctx*>(&slot);  // only passed to the stubs
  int cases = 0;
  {
    dlsm_adapter::FullFilterBlockBuilder b(&mr, 10, fake_ctx, opt);
    if (run(b, cases)) return 1;
  }
  {
    MrShaped ibv{nullptr, nullptr, slot.data(), slot.size(), 0, 0, 0};
    dlsm_adapter::FullFilterBlockBuilder b(&ibv, 10);
    if (run(b, cases)) return 1;
    CHECK(b.result.data() == slot.data());
  }
  std::printf("OK adapter addkey cpu (%d cases, avx512 %d)\n", cases, dlsm_adapter::HasAvx512() ? 1 : 0);
  return 0;
}
