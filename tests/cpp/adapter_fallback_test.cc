// GPU test of the adapter's reference-signature surface and its failure path
// (include/dlsm_bloom_adapter.hpp), against the oracle (test infrastructure).
// Built and run by tests/test_gpu_adapter.py.
//
//  1. FullFilterBlockBuilder(ibv_mr*, int) (table/full_filter_block.h:35) with
//     an injected device failure (DLSM_OPT_FAULT_INJECT: DLSM_E_DEVICE,
//     DLSM_E_NOMEM) at 0, 1, 7 and 153,846 keys: Finish re-runs the reference
//     loop on the host and the filter equals the oracle's -- never the 0-byte
//     filter the reference reader (full_filter_block.cc:191-249) would exit
//     on; the context's and the process's fallback counters record each one.
//     The same for the adapter's other constructor (keys over PCIe, hashes,
//     mixed lengths), a too-small slot (the match-everything filter), and the
//     legacy FilterBlockBuilder / BloomFilterPolicy::CreateFilter.
//  2. FullFilterBlockReader(const Slice&, shared_ptr<Manager>, FilterSide)
//     (full_filter_block.h:76-77) and NewBloomFilterPolicy(int)
//     (filter_policy.h:71): single-key KeyMayMatch on the host, no device
//     allocation until the first batch; KeysMayMatch on the GPU (and on the
//     host under an injected fault); a Compute-side reader frees its slot
//     through the manager, a Memory-side one does not.
//  3. Single-key KeyMayMatch latency in ns (one JSON line).
// Without a visible device (the CPU suite) the same program checks the
// no-device path: every build and batch falls back to the host loops, with
// the same bytes and answers, and each fallback is counted.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "dlsm_bloom_adapter.hpp"

extern "C" {
int64_t orc_full_build(const uint8_t*, const uint64_t*, uint32_t, uint64_t, int, uint8_t*, uint64_t);
int orc_full_key_may_match(const uint8_t*, uint64_t, const uint8_t*, size_t);
int64_t orc_legacy_build(const uint8_t*, const uint64_t*, uint32_t, uint64_t, int, uint8_t*, uint64_t);
int orc_legacy_key_may_match(const uint8_t*, uint64_t, const uint8_t*, size_t);
void orc_dbbench_key(uint64_t v, int key_size, uint8_t* out);
int64_t orc_filter_block_build(const uint8_t*, const uint64_t*, uint32_t, uint64_t, const uint64_t*,
                               const uint64_t*, int, int, int, uint8_t*, uint64_t);
int orc_filter_block_key_may_match(const uint8_t*, uint64_t, uint64_t, const uint8_t*, size_t, int);
}

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);      \
      return 1;                                                    \
    }                                                              \
  } while (0)

using dlsm_adapter::Slice;

struct IbvMrShaped {  // <infiniband/verbs.h> struct ibv_mr's fields
  void* context;
  void* pd;
  void* addr;
  size_t length;
  uint32_t handle, lkey, rkey;
};

// util/rdma.h:75's Chunk_type and the one RDMA_Manager method a reader calls
// (util/rdma.h:411), counting the slots it is handed back.
enum Chunk_type { Message = 1, Version_edit = 2, IndexChunk = 3, IndexChunk_Small = 4, FilterChunk = 5 };
struct MockRdmaManager {
  int freed = 0;
  const void* last = nullptr;
  Chunk_type last_type = Message;
  bool Deallocate_Local_RDMA_Slot(void* p, Chunk_type t) {
    freed++;
    last = p;
    last_type = t;
    return true;
  }
};
enum class HostFilterSide { Compute, Memory };  // the reference's enum, declared by the host

static bool g_dev = false;  // a device is visible: faults are injected, GPU answers expected

// DLSM_OPT_FAULT_INJECT on a context (a no-op without a device: every call fails anyway)
static int inject(dlsm_ctx* ctx, int v) { return ctx ? dlsm_ctx_set_option(ctx, DLSM_OPT_FAULT_INJECT, v) : DLSM_OK; }

static uint64_t process_fallbacks() {
  uint64_t n = 0;
  dlsm_fallback_stats(nullptr, nullptr, &n);
  return n;
}

struct KeySet {
  std::string flat;
  std::vector<uint64_t> offs{0};
  void add(const char* p, size_t n) {
    flat.append(p, n);
    offs.push_back(flat.size());
  }
  size_t n() const { return offs.size() - 1; }
  Slice at(size_t i) const { return Slice(flat.data() + offs[i], offs[i + 1] - offs[i]); }
};

static KeySet table_keys(int n, int shape) {
  KeySet ks;
  uint32_t x = 12345u + shape;
  for (int i = 0; i < n; i++) {
    uint8_t k[20];
    orc_dbbench_key(static_cast<uint64_t>(i / (i % 5 == 0 ? 2 : 1)) * 7 + 3, 20, k);  // runs of repeats
    int len = 20;
    if (shape == 1) {  // mixed lengths, bytes >= 0x80 in the tails
      x = x * 1664525u + 1013904223u;
      len = 1 + static_cast<int>(x >> 28);
      k[len - 1] = static_cast<uint8_t>(x >> 8);
    }
    ks.add(reinterpret_cast<char*>(k), len);
  }
  return ks;
}

static int full_build_fallbacks() {
  dlsm_ctx* tctx = nullptr;
  CHECK((dlsm_thread_ctx(&tctx) == DLSM_OK && tctx) == g_dev);
  std::vector<char> slot(256 * 1024);
  IbvMrShaped mr{nullptr, nullptr, slot.data(), slot.size(), 0, 0, 0};
  for (int fault : {4, 5}) {  // DLSM_E_DEVICE, DLSM_E_NOMEM
    for (int n : {0, 1, 7, 153846}) {
      const KeySet ks = table_keys(n, 0);
      std::vector<uint8_t> want(slot.size());
      const int64_t wl = orc_full_build(reinterpret_cast<const uint8_t*>(ks.flat.data()), ks.offs.data(), 0, ks.n(),
                                        10, want.data(), want.size());
      CHECK(wl > 0);
      // (a) the reference's own signature; the thread context fails
      std::memset(slot.data(), 0x5a, slot.size());  // a dirty slot: every byte must be written
      dlsm_adapter::FullFilterBlockBuilder b(&mr, 10);
      b.RestartBlock(0);
      for (size_t i = 0; i < ks.n(); i++) b.AddKey(ks.at(i));
      uint64_t c0 = 0, p0 = process_fallbacks();
      dlsm_fallback_stats(tctx, &c0, nullptr);
      CHECK(inject(tctx, fault) == DLSM_OK);
      b.Finish();
      CHECK(inject(tctx, 0) == DLSM_OK);
      uint64_t c1 = 0;
      dlsm_fallback_stats(tctx, &c1, nullptr);
      CHECK(b.status() == DLSM_OK && b.device_status() == (g_dev ? -fault : DLSM_E_DEVICE) && b.fell_back());
      CHECK(c1 == c0 + (g_dev ? 1u : 0u) && process_fallbacks() == p0 + 1);
      CHECK(static_cast<int64_t>(b.result.size()) == wl && b.result.data() == slot.data());
      CHECK(std::memcmp(b.result.data(), want.data(), wl) == 0);
      if (!g_dev) continue;
      // the next table on the healthy context runs on the GPU again
      b.Reset();
      for (size_t i = 0; i < ks.n(); i++) b.AddKey(ks.at(i));
      b.Finish();
      CHECK(b.status() == DLSM_OK && b.device_status() == DLSM_OK && !b.fell_back());
      CHECK(static_cast<int64_t>(b.result.size()) == wl && std::memcmp(b.result.data(), want.data(), wl) == 0);
    }
  }
  // (b) the adapter's constructor on an explicit context: raw keys (fixed and
  // mixed lengths), host hashes, and through a batcher whose executor fails
  dlsm_ctx* ctx = nullptr;
  CHECK((dlsm_ctx_create(0, &ctx) == DLSM_OK) == g_dev);
  for (int shape = 0; shape < 2; shape++) {
    for (int hashed = 0; hashed < 2; hashed++) {
      const KeySet ks = table_keys(40000, shape);
      std::vector<uint8_t> want(slot.size());
      const int64_t wl = orc_full_build(reinterpret_cast<const uint8_t*>(ks.flat.data()), ks.offs.data(), 0, ks.n(),
                                        10, want.data(), want.size());
      dlsm_adapter::FilterSlot fs{slot.data(), slot.size()};
      dlsm_adapter::BuilderOptions opt;
      opt.hash_in_addkey = hashed == 1;
      dlsm_adapter::FullFilterBlockBuilder b(&fs, 10, ctx, opt);
      for (size_t i = 0; i < ks.n(); i++) b.AddKey(ks.at(i));
      std::memset(slot.data(), 0x77, slot.size());
      CHECK(inject(ctx, 4) == DLSM_OK);
      b.Finish();
      CHECK(inject(ctx, 0) == DLSM_OK);
      CHECK(b.status() == DLSM_OK && b.fell_back());
      CHECK(static_cast<int64_t>(b.result.size()) == wl && std::memcmp(b.result.data(), want.data(), wl) == 0);
    }
  }
  // (c) a slot too small for the filter: the match-everything filter, which
  // the reference reader accepts and which answers true for every key
  {
    std::vector<char> small(4096, 0x11);
    IbvMrShaped smr{nullptr, nullptr, small.data(), small.size(), 0, 0, 0};
    dlsm_adapter::FullFilterBlockBuilder b(&smr, 10);
    const KeySet ks = table_keys(10000, 0);
    for (size_t i = 0; i < ks.n(); i++) b.AddKey(ks.at(i));
    b.Finish();
    CHECK(b.status() == DLSM_E_CAPACITY && b.result.size() == 69 && b.fell_back() == !g_dev);
    dlsm_adapter::FullFilterBlockReader r(b.result, nullptr);
    CHECK(r.status() == DLSM_OK && r.num_lines() == 1);
    for (int q = 0; q < 1000; q++) {
      uint8_t k[20];
      orc_dbbench_key(static_cast<uint64_t>(q) * 13 + 1, 20, k);
      CHECK(r.KeyMayMatch(Slice(reinterpret_cast<char*>(k), 20)));
      CHECK(orc_full_key_may_match(reinterpret_cast<const uint8_t*>(small.data()), 69, k, 20) == 1);
    }
  }
  // (d) legacy: BloomFilterPolicy::CreateFilter and FilterBlockBuilder::Finish
  {
    const dlsm_adapter::FilterPolicy* pol = dlsm_adapter::NewBloomFilterPolicy(10, ctx);
    const KeySet ks = table_keys(3000, 1);
    std::vector<Slice> keys;
    for (size_t i = 0; i < ks.n(); i++) keys.push_back(ks.at(i));
    std::vector<uint8_t> want(8192);
    const int64_t wl = orc_legacy_build(reinterpret_cast<const uint8_t*>(ks.flat.data()), ks.offs.data(), 0, ks.n(),
                                        10, want.data(), want.size());
    std::vector<char> buf(16384, 0x3c);
    Slice dst(buf.data(), 0);
    dst.append("pre", 3);
    CHECK(inject(ctx, 5) == DLSM_OK);
    const uint64_t p0 = process_fallbacks();
    pol->CreateFilter(keys.data(), static_cast<int>(keys.size()), &dst);
    CHECK(process_fallbacks() == p0 + 1);
    CHECK(static_cast<int64_t>(dst.size()) == 3 + wl && std::memcmp(dst.data() + 3, want.data(), wl) == 0);

    std::vector<char> fslot(64 * 1024, 0x42);
    dlsm_adapter::FilterSlot mr2{fslot.data(), fslot.size()};
    dlsm_adapter::FilterBlockBuilder fb(&mr2, 10, ctx);
    KeySet fk;
    std::vector<uint64_t> ke{0}, eo{0}, kblock;
    uint64_t off = 0;
    fb.StartBlock(0);
    for (int blk = 0; blk < 30; blk++) {
      for (int i = 0; i < 5 + (blk * 7) % 11; i++) {
        uint8_t k[20];
        orc_dbbench_key(500 * blk + i, 20, k);
        fk.add(reinterpret_cast<char*>(k), 20);
        kblock.push_back(off);
        fb.AddKey(fk.at(fk.n() - 1));
      }
      off += 900 + 1700 * (blk % 4);  // some blocks span several 2 KiB ranges
      fb.StartBlock(off);
      ke.push_back(fk.n());
      eo.push_back(off);
    }
    for (int i = 0; i < 9; i++) {  // keys after the last block end: Finish's filter
      uint8_t k[20];
      orc_dbbench_key(900000 + i, 20, k);
      fk.add(reinterpret_cast<char*>(k), 20);
      fb.AddKey(fk.at(fk.n() - 1));
    }
    const uint64_t p1 = process_fallbacks();
    Slice blk = fb.Finish();
    CHECK(inject(ctx, 0) == DLSM_OK);
    CHECK(fb.status() == DLSM_OK && process_fallbacks() == p1 + 1);
    std::vector<uint8_t> wb(64 * 1024);
    const int64_t wbl = orc_filter_block_build(reinterpret_cast<const uint8_t*>(fk.flat.data()), fk.offs.data(), 0,
                                               fk.n(), ke.data(), eo.data(), static_cast<int>(ke.size()), 0, 10,
                                               wb.data(), wb.size());
    CHECK(wbl > 0 && static_cast<int64_t>(blk.size()) == wbl && std::memcmp(blk.data(), wb.data(), wbl) == 0);
    dlsm_adapter::FilterBlockReader rd(blk, ctx);
    for (size_t i = 0; i < kblock.size(); i++)
      CHECK(rd.KeyMayMatch(kblock[i], fk.at(i)) ==
            (orc_filter_block_key_may_match(wb.data(), wbl, kblock[i],
                                            reinterpret_cast<const uint8_t*>(fk.at(i).data()), 20, 0) != 0));
    delete pol;
  }
  dlsm_ctx_destroy(ctx);
  return 0;
}

static int reference_readers() {
  dlsm_ctx* tctx = nullptr;
  CHECK((dlsm_thread_ctx(&tctx) == DLSM_OK && tctx) == g_dev);
  // one 1.6 M-key filter (config 2's table) in a slot the manager owns
  const int n = 1600000;
  KeySet ks;
  for (int i = 0; i < n; i++) {
    uint8_t k[20];
    orc_dbbench_key(static_cast<uint64_t>(i) * 2, 20, k);
    ks.add(reinterpret_cast<char*>(k), 20);
  }
  std::vector<uint8_t> filt(2100000);
  const int64_t fl = orc_full_build(reinterpret_cast<const uint8_t*>(ks.flat.data()), nullptr, 20, n, 10,
                                    filt.data(), filt.size());
  CHECK(fl == 2000069);
  auto mgr = std::make_shared<MockRdmaManager>();
  const Slice contents(reinterpret_cast<const char*>(filt.data()), static_cast<size_t>(fl));
  const int nq = 2000000;
  std::vector<std::string> qs;
  qs.reserve(nq);
  for (int i = 0; i < nq; i++) {
    uint8_t k[20];
    orc_dbbench_key(static_cast<uint64_t>(i) * 3 + 1, 20, k);  // 26.7 % present
    qs.emplace_back(reinterpret_cast<char*>(k), 20);
  }
  double ns_per_key = 0;
  {
    dlsm_adapter::FullFilterBlockReader r(contents, mgr, HostFilterSide::Compute);
    CHECK(r.status() == DLSM_OK && r.num_probes() == 6 && r.num_lines() == 31251);
    // single keys: host, oracle-equal, no device copy
    for (int i = 0; i < nq; i += 7)
      CHECK(r.KeyMayMatch(Slice(qs[i])) ==
            (orc_full_key_may_match(filt.data(), fl, reinterpret_cast<const uint8_t*>(qs[i].data()), 20) == 1));
    for (int i = 0; i < n; i += 97) CHECK(r.KeyMayMatch(ks.at(i)));
    CHECK(!r.device_resident());
    // latency: one key at a time, as Table::InternalGet calls it
    size_t hits = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < nq; i++) hits += r.KeyMayMatch(Slice(qs[i])) ? 1 : 0;
    const auto t1 = std::chrono::steady_clock::now();
    ns_per_key = std::chrono::duration<double, std::nano>(t1 - t0).count() / nq;
    CHECK(hits > static_cast<size_t>(nq) / 4);  // 26.7 % present, ~1 % false positives
    // a batch: GPU, oracle-equal; the device copy appears now
    std::vector<Slice> q;
    for (int i = 0; i < 300000; i++) q.emplace_back(qs[i]);
    std::vector<uint8_t> got(q.size(), 9);
    const uint64_t p0 = process_fallbacks();
    CHECK(r.KeysMayMatch(q.data(), q.size(), got.data()) == DLSM_OK);
    if (g_dev) CHECK(r.last_device_status() == DLSM_OK && r.device_resident() && process_fallbacks() == p0);
    else CHECK(r.last_device_status() == DLSM_E_DEVICE && !r.device_resident() && process_fallbacks() == p0 + 1);
    for (size_t i = 0; i < q.size(); i++)
      CHECK(got[i] == orc_full_key_may_match(filt.data(), fl, reinterpret_cast<const uint8_t*>(q[i].data()), 20));
    // the same batch under an injected device failure: host answers, counted
    const uint64_t p1 = process_fallbacks();
    CHECK(inject(tctx, 4) == DLSM_OK);
    std::fill(got.begin(), got.end(), 9);
    CHECK(r.KeysMayMatch(q.data(), q.size(), got.data()) == DLSM_OK);
    CHECK(inject(tctx, 0) == DLSM_OK);
    CHECK(r.last_device_status() == DLSM_E_DEVICE && process_fallbacks() == p1 + 1);
    for (size_t i = 0; i < q.size(); i++)
      CHECK(got[i] == orc_full_key_may_match(filt.data(), fl, reinterpret_cast<const uint8_t*>(q[i].data()), 20));
    CHECK(mgr->freed == 0);
  }
  CHECK(mgr->freed == 1 && mgr->last == filt.data() && mgr->last_type == FilterChunk);  // Compute side frees
  {
    dlsm_adapter::FullFilterBlockReader r(contents, mgr, HostFilterSide::Memory);
    CHECK(r.KeyMayMatch(ks.at(5)));
  }
  CHECK(mgr->freed == 1);  // Memory side does not
  // the reference reader's log2_cache_line_size_ == 0 branch (len % L == 0,
  // L * 64 != len): one-byte "lines"
  {
    std::vector<uint8_t> odd(3 * 10 + 5, 0);
    for (size_t i = 0; i < 30; i++) odd[i] = static_cast<uint8_t>(0x5b * i + 17);
    odd[30] = 3;
    odd[31] = 10;  // L = 10, len 30
    const Slice oc(reinterpret_cast<const char*>(odd.data()), odd.size());
    dlsm_adapter::FullFilterBlockReader r(oc, mgr, dlsm_adapter::Memory);
    CHECK(r.status() == DLSM_OK);
    for (int i = 0; i < 5000; i++)
      CHECK(r.KeyMayMatch(Slice(qs[i])) ==
            (orc_full_key_may_match(odd.data(), odd.size(), reinterpret_cast<const uint8_t*>(qs[i].data()), 20) == 1));
  }
  // NewBloomFilterPolicy(int): the reference's signature (db_bench.cc:638)
  {
    const dlsm_adapter::FilterPolicy* pol = dlsm_adapter::NewBloomFilterPolicy(10);
    const KeySet lk = table_keys(20000, 1);
    std::vector<Slice> keys;
    for (size_t i = 0; i < lk.n(); i++) keys.push_back(lk.at(i));
    std::vector<char> buf(64 * 1024, 0x19);
    Slice dst(buf.data(), 0);
    const uint64_t p0 = process_fallbacks();
    pol->CreateFilter(keys.data(), static_cast<int>(keys.size()), &dst);
    CHECK(process_fallbacks() == p0 + (g_dev ? 0u : 1u));
    std::vector<uint8_t> want(64 * 1024);
    const int64_t wl = orc_legacy_build(reinterpret_cast<const uint8_t*>(lk.flat.data()), lk.offs.data(), 0, lk.n(),
                                        10, want.data(), want.size());
    CHECK(static_cast<int64_t>(dst.size()) == wl && std::memcmp(dst.data(), want.data(), wl) == 0);
    for (int i = 0; i < 100000; i++) {
      const Slice q(qs[i]);
      CHECK(pol->KeyMayMatch(q, dst) ==
            (orc_legacy_key_may_match(want.data(), wl, reinterpret_cast<const uint8_t*>(q.data()), 20) != 0));
    }
    // legacy edge answers (util/bloom.cc:59,67-70): len < 2 false, k > 30 true
    CHECK(!pol->KeyMayMatch(Slice("a", 1), Slice("\x06", 1)));
    const char big_k[3] = {0, 0, 31};
    CHECK(pol->KeyMayMatch(Slice("a", 1), Slice(big_k, 3)));
    const char neg_k[3] = {0, 0, static_cast<char>(-3)};
    CHECK(pol->KeyMayMatch(Slice("a", 1), Slice(neg_k, 3)));
    delete pol;
  }
  std::printf("{\"single_key_ns\": %.1f, \"filter_keys\": %d, \"lookups\": %d, \"device\": %s}\n", ns_per_key, n,
              nq, g_dev ? "true" : "false");
  return 0;
}

// dLSM starts a std::thread per subcompaction (db/db_impl.cc:3373-3386):
// 12 rounds of 4 short-lived threads, one reference-signature build each.
// Contexts come back to the free list at thread exit and the next threads
// take them: at most 4 are created for these 48 threads.
static int short_lived_threads() {
  uint64_t c0 = 0, r0 = 0, i0 = 0;
  CHECK(dlsm_thread_ctx_stats(&c0, &r0, &i0) == DLSM_OK);
  const KeySet ks = table_keys(153846, 0);
  std::vector<uint8_t> want(256 * 1024);
  const int64_t wl = orc_full_build(reinterpret_cast<const uint8_t*>(ks.flat.data()), ks.offs.data(), 0, ks.n(), 10,
                                    want.data(), want.size());
  int bad = 0;
  for (int round = 0; round < 12; round++) {
    std::vector<std::thread> th;
    std::vector<std::vector<char>> slots(4, std::vector<char>(256 * 1024));
    for (int t = 0; t < 4; t++)
      th.emplace_back([&, t] {
        IbvMrShaped mr{nullptr, nullptr, slots[t].data(), slots[t].size(), 0, 0, 0};
        dlsm_adapter::FullFilterBlockBuilder b(&mr, 10);
        for (size_t i = 0; i < ks.n(); i++) b.AddKey(ks.at(i));
        b.Finish();
        if (b.status() != DLSM_OK || b.fell_back() || static_cast<int64_t>(b.result.size()) != wl ||
            std::memcmp(b.result.data(), want.data(), wl) != 0)
          __atomic_add_fetch(&bad, 1, __ATOMIC_RELAXED);
      });
    for (auto& x : th) x.join();
  }
  uint64_t c1 = 0, r1 = 0, i1 = 0;
  CHECK(dlsm_thread_ctx_stats(&c1, &r1, &i1) == DLSM_OK);
  CHECK(bad == 0);
  CHECK(c1 - c0 <= 4 && (c1 - c0) + (r1 - r0) == 48 && i1 >= 4);
  std::printf("{\"short_lived_threads\": 48, \"contexts_created\": %llu, \"reused\": %llu}\n",
              static_cast<unsigned long long>(c1 - c0), static_cast<unsigned long long>(r1 - r0));
  return 0;
}

int main() {
  int nd = 0;
  g_dev = dlsm_device_count(&nd) == DLSM_OK && nd > 0;
  if (process_fallbacks() != 0) return 2;
  if (reference_readers() != 0) return 1;
  if (full_build_fallbacks() != 0) return 1;
  if (g_dev && short_lived_threads() != 0) return 1;
  std::printf("OK adapter fallback\n");
  return 0;
}
