// GPU test of the C++ adapter (include/dlsm_bloom_adapter.hpp) -- the classes a
// reference TableBuilder / Table would call -- against the oracle (test
// infrastructure).  Built and run by tests/test_gpu_adapter.py.
#include <cstdio>
#include <cstring>
#include <string>
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

// <infiniband/verbs.h>'s struct ibv_mr field layout: the reference-signature
// constructor reads addr and length only, so an ibv_mr binds as-is.
struct IbvMrShaped {
  void* context;
  void* pd;
  void* addr;
  size_t length;
  uint32_t handle, lkey, rkey;
};

// FullFilterBlockBuilder(ibv_mr* mr, int bloombits_per_key) -- the reference's
// own signature (table/full_filter_block.h:35) and AddKey
// (full_filter_block.cc:39-49), the thread's context: every filter byte vs the
// oracle, in a page-locked slot (kernels store straight into it) and in a
// pageable one, with repeated keys (the dedup), Move_buffer and Reset.
static int reference_signature() {
  void* pinned = nullptr;
  CHECK(dlsm_host_alloc(256 * 1024, &pinned) == DLSM_OK);
  std::vector<char> pageable(256 * 1024, 0);
  for (int slot_kind = 0; slot_kind < 2; slot_kind++) {
    char* base = slot_kind ? pageable.data() : static_cast<char*>(pinned);
    IbvMrShaped mr{nullptr, nullptr, base, 256 * 1024, 0, 0, 0};
    for (int n : {0, 1, 7, 4097, 153846}) {
      std::memset(base, 0, 256 * 1024);
      dlsm_adapter::FullFilterBlockBuilder b(&mr, 10);
      b.RestartBlock(0);
      std::string flat;
      std::vector<uint64_t> offs{0};
      for (int i = 0; i < n; i++) {
        uint8_t k[20];
        orc_dbbench_key(static_cast<uint64_t>(i / (i % 5 == 0 ? 2 : 1)) * 7 + 3, 20, k);  // runs of repeats
        b.AddKey(Slice(reinterpret_cast<char*>(k), 20));
        flat.append(reinterpret_cast<char*>(k), 20);
        offs.push_back(flat.size());
      }
      b.Finish();
      CHECK(b.status() == DLSM_OK);
      std::vector<uint8_t> want(256 * 1024, 0);
      const int64_t wl = orc_full_build(reinterpret_cast<const uint8_t*>(flat.data()), offs.data(), 0, n, 10,
                                        want.data(), want.size());
      CHECK(wl > 0 && static_cast<int64_t>(b.result.size()) == wl);
      CHECK(b.result.data() == base);
      CHECK(std::memcmp(b.result.data(), want.data(), wl) == 0);
      // a second table through the same builder after Move_buffer into the slot's back half
      b.Move_buffer(base + 128 * 1024);
      b.RestartBlock(0);
      for (int i = 0; i < 1000; i++) {
        uint8_t k[20];
        orc_dbbench_key(static_cast<uint64_t>(i) + 99, 20, k);
        b.AddKey(Slice(reinterpret_cast<char*>(k), 20));
      }
      b.Finish();
      CHECK(b.status() == DLSM_OK && b.result.data() == base + 128 * 1024);
      std::string f2;
      std::vector<uint64_t> o2{0};
      for (int i = 0; i < 1000; i++) {
        uint8_t k[20];
        orc_dbbench_key(static_cast<uint64_t>(i) + 99, 20, k);
        f2.append(reinterpret_cast<char*>(k), 20);
        o2.push_back(f2.size());
      }
      const int64_t w2 = orc_full_build(reinterpret_cast<const uint8_t*>(f2.data()), o2.data(), 0, 1000, 10,
                                        want.data(), want.size());
      CHECK(static_cast<int64_t>(b.result.size()) == w2 && std::memcmp(b.result.data(), want.data(), w2) == 0);
      b.Reset();
      CHECK(b.result.size() == 0 && b.result.data() == base);
    }
  }
  // the context came from the thread (dlsm_thread_ctx), the same one every time
  dlsm_ctx* t1 = nullptr;
  dlsm_ctx* t2 = nullptr;
  CHECK(dlsm_thread_ctx(&t1) == DLSM_OK && dlsm_thread_ctx(&t2) == DLSM_OK && t1 && t1 == t2);
  CHECK(dlsm_host_free(pinned) == DLSM_OK);
  return 0;
}

int main() {
  if (reference_signature() != 0) return 1;
  dlsm_ctx* ctx = nullptr;
  CHECK(dlsm_ctx_create(0, &ctx) == DLSM_OK);
  // ---- FullFilterBlockBuilder: the TableBuilder call shape ----
  for (int n : {0, 1, 52, 5000, 153846}) {
    std::vector<char> slot(256 * 1024, 0);  // FilterChunk slot (options.h:28), zeroed
    dlsm_adapter::FilterSlot mr{slot.data(), slot.size()};
    dlsm_adapter::FullFilterBlockBuilder b(&mr, 10, ctx);
    b.RestartBlock(0);
    std::string flat;
    std::vector<uint64_t> offs{0};
    for (int i = 0; i < n; i++) {
      uint8_t k[20];
      orc_dbbench_key(static_cast<uint64_t>(i) * 3 + 1, 20, k);
      b.AddKey(Slice(reinterpret_cast<char*>(k), 20));
      flat.append(reinterpret_cast<char*>(k), 20);
      offs.push_back(flat.size());
    }
    b.Finish();
    CHECK(b.status() == DLSM_OK);
    std::vector<uint8_t> want(256 * 1024, 0);
    int64_t wl = orc_full_build(reinterpret_cast<const uint8_t*>(flat.data()), offs.data(), 0, n, 10,
                                want.data(), want.size());
    CHECK(wl > 0 && static_cast<int64_t>(b.result.size()) == wl);
    CHECK(std::memcmp(b.result.data(), want.data(), wl) == 0);
    CHECK(b.result.data() == slot.data());
    // ---- FullFilterBlockReader ----
    if (n > 0) {
      dlsm_adapter::FullFilterBlockReader r(b.result, ctx);
      CHECK(r.status() == DLSM_OK && r.num_probes() == 6);
      std::vector<Slice> q;
      std::vector<std::string> qs;
      for (int i = 0; i < 3000; i++) {
        uint8_t k[20];
        orc_dbbench_key(static_cast<uint64_t>(i), 20, k);
        qs.emplace_back(reinterpret_cast<char*>(k), 20);
      }
      for (auto& s : qs) q.emplace_back(s);
      std::vector<uint8_t> got(q.size());
      CHECK(r.KeysMayMatch(q.data(), q.size(), got.data()) == DLSM_OK);
      for (size_t i = 0; i < q.size(); i++)
        CHECK(got[i] == orc_full_key_may_match(want.data(), wl,
                                               reinterpret_cast<const uint8_t*>(q[i].data()), 20));
      CHECK(r.KeyMayMatch(Slice(flat.data(), 20)));
    }
    b.Reset();
    CHECK(b.result.size() == 0);
  }
  // corrupt filter -> status, not exit(1)
  {
    char bad[69] = {0};
    bad[65] = 1;  // k byte 0
    dlsm_adapter::FullFilterBlockReader r(Slice(bad, sizeof(bad)), ctx);
    CHECK(r.status() == DLSM_E_CORRUPT);
    CHECK(r.KeyMayMatch(Slice("x", 1)));  // errors are potential matches
  }
  // ---- BloomFilterPolicy (legacy format) ----
  {
    dlsm_adapter::BloomFilterPolicy pol(10, ctx);
    CHECK(std::strcmp(pol.Name(), "TimberSaw.BuiltinBloomFilter2") == 0);
    std::vector<char> buf(64 * 1024, 0);
    Slice dst(buf.data(), 0);
    const char* prefix = "hdr";
    dst.append(prefix, 3);  // CreateFilter appends after existing content
    std::vector<std::string> ks = {"hello", "world", "", "a", "0123456789abcdef0123"};
    std::vector<Slice> keys(ks.begin(), ks.end());
    pol.CreateFilter(keys.data(), static_cast<int>(keys.size()), &dst);
    CHECK(pol.status() == DLSM_OK);
    std::string flat;
    std::vector<uint64_t> offs{0};
    for (auto& s : ks) {
      flat += s;
      offs.push_back(flat.size());
    }
    std::vector<uint8_t> want(1024, 0);
    int64_t wl = orc_legacy_build(reinterpret_cast<const uint8_t*>(flat.data()), offs.data(), 0,
                                  ks.size(), 10, want.data(), want.size());
    CHECK(static_cast<int64_t>(dst.size()) == 3 + wl);
    CHECK(std::memcmp(dst.data(), "hdr", 3) == 0);
    CHECK(std::memcmp(dst.data() + 3, want.data(), wl) == 0);
    Slice filt(dst.data() + 3, wl);
    for (auto& s : ks) CHECK(pol.KeyMayMatch(Slice(s), filt));
    for (const char* q : {"x", "foo", "hello!", "zz"})
      CHECK(pol.KeyMayMatch(Slice(q, std::strlen(q)), filt) ==
            (orc_legacy_key_may_match(want.data(), wl, reinterpret_cast<const uint8_t*>(q),
                                      std::strlen(q)) != 0));
  }
  // ---- FilterPolicy surface through base-class pointers (Options::filter_policy):
  // NewBloomFilterPolicy, and InternalFilterPolicy over internal keys, both the
  // GPU form (suffix_len 8 on the device) and the generic wrapper form ----
  {
    const dlsm_adapter::FilterPolicy* user = dlsm_adapter::NewBloomFilterPolicy(10, ctx);
    dlsm_adapter::BloomFilterPolicy gpu_user(10, ctx);
    dlsm_adapter::InternalFilterPolicy ip_gpu(&gpu_user);
    dlsm_adapter::InternalFilterPolicy ip_wrap(user);  // any FilterPolicy: host-side ExtractUserKey
    const dlsm_adapter::FilterPolicy* policies[3] = {user, &ip_gpu, &ip_wrap};
    const bool internal[3] = {false, true, true};
    std::vector<std::string> uk;
    for (int i = 0; i < 3000; i++) {
      uint8_t k[20];
      orc_dbbench_key(static_cast<uint64_t>(i) * 7 + 3, 20, k);
      uk.emplace_back(reinterpret_cast<char*>(k), 20);
    }
    uk.push_back("");      // empty user key
    uk.push_back("x");     // 1-byte tail (sign-extended bytes live in the fixtures)
    std::string flat;
    std::vector<uint64_t> offs{0};
    for (auto& s : uk) {
      flat += s;
      offs.push_back(flat.size());
    }
    std::vector<uint8_t> want(8192, 0);
    const int64_t wl = orc_legacy_build(reinterpret_cast<const uint8_t*>(flat.data()), offs.data(), 0,
                                        uk.size(), 10, want.data(), want.size());
    CHECK(wl > 0);
    for (int p = 0; p < 3; p++) {
      const dlsm_adapter::FilterPolicy* pol = policies[p];
      CHECK(std::strcmp(pol->Name(), "TimberSaw.BuiltinBloomFilter2") == 0);
      std::vector<std::string> ks;  // user keys, or internal keys user||Fixed64(seq<<8|type)
      for (size_t i = 0; i < uk.size(); i++) {
        std::string k = uk[i];
        if (internal[p]) {
          const uint64_t tag = (static_cast<uint64_t>(1000 + i) << 8) | 1u;
          k.append(reinterpret_cast<const char*>(&tag), 8);  // little-endian host
        }
        ks.push_back(k);
      }
      std::vector<Slice> keys(ks.begin(), ks.end());
      std::vector<char> buf(16 * 1024, 0);
      Slice dst(buf.data(), 0);
      dst.append("ab", 2);
      pol->CreateFilter(keys.data(), static_cast<int>(keys.size()), &dst);
      CHECK(static_cast<int64_t>(dst.size()) == 2 + wl);
      CHECK(std::memcmp(dst.data() + 2, want.data(), wl) == 0);
      if (internal[p])  // the reference rewrites keys[] to the user keys (dbformat.cc:97-101)
        for (size_t i = 0; i < keys.size(); i++) CHECK(keys[i].size() == uk[i].size() && keys[i].data() == ks[i].data());
      Slice filt(dst.data() + 2, wl);
      for (size_t i = 0; i < ks.size(); i += 7) CHECK(pol->KeyMayMatch(Slice(ks[i]), filt));
      for (int q = 0; q < 2000; q++) {
        uint8_t k[28];
        orc_dbbench_key(static_cast<uint64_t>(q) * 7 + 5, 20, k);  // mostly absent
        const uint64_t tag = (static_cast<uint64_t>(q) << 8) | 1u;
        std::memcpy(k + 20, &tag, 8);
        const bool got = pol->KeyMayMatch(Slice(reinterpret_cast<char*>(k), internal[p] ? 28 : 20), filt);
        CHECK(got == (orc_legacy_key_may_match(want.data(), wl, k, 20) != 0));
      }
    }
    delete user;
  }
  // ---- FullFilterBlockBuilder: repeated user keys (several versions of a key
  // in a compaction output) lower the line count; the builder asks for the
  // exact count; keys of mixed length take the offsets path ----
  {
    std::vector<char> slot(256 * 1024, 0);
    dlsm_adapter::FilterSlot mr{slot.data(), slot.size()};
    dlsm_adapter::FullFilterBlockBuilder b(&mr, 10, ctx);
    for (int mixed = 0; mixed < 2; mixed++) {
      std::string flat;
      std::vector<uint64_t> offs{0};
      b.RestartBlock(0);
      for (int i = 0; i < 60000; i++) {
        uint8_t k[20];
        orc_dbbench_key(static_cast<uint64_t>(i / 3), 20, k);  // 3 versions per user key
        const int len = mixed ? 12 + (i / 3) % 9 : 20;
        b.AddKey(Slice(reinterpret_cast<char*>(k), len));
        flat.append(reinterpret_cast<char*>(k), len);
        offs.push_back(flat.size());
      }
      b.Finish();
      CHECK(b.status() == DLSM_OK);
      std::vector<uint8_t> want(256 * 1024, 0);
      const int64_t wl = orc_full_build(reinterpret_cast<const uint8_t*>(flat.data()), offs.data(), 0, 60000, 10,
                                        want.data(), want.size());
      uint32_t L60k = 0;
      uint64_t n60k = 0;
      dlsm_bloom_full_size(60000, 10, &L60k, &n60k);
      CHECK(wl > 0 && static_cast<uint64_t>(wl) < n60k && static_cast<int64_t>(b.result.size()) == wl);
      CHECK(std::memcmp(b.result.data(), want.data(), wl) == 0);
      b.Reset();
    }
  }
  // ---- FilterBlockBuilder / FilterBlockReader: TableBuilder's call shape
  // (StartBlock after each data block flush, filter_block.cc:32-38) ----
  {
    std::vector<char> slot(64 * 1024, 0);
    dlsm_adapter::FilterSlot mr{slot.data(), slot.size()};
    dlsm_adapter::FilterBlockBuilder fb(&mr, 10, ctx);
    std::vector<std::string> ks;
    std::vector<uint64_t> ke, eo, key_block;
    uint64_t off = 0;
    fb.StartBlock(0);  // TableBuilder ctor
    ke.push_back(0);
    eo.push_back(0);
    for (int b = 0; b < 40; b++) {
      for (int i = 0; i < 7 + (b * 5) % 13; i++) {
        char k[20];
        orc_dbbench_key(1000 * b + i, 20, reinterpret_cast<uint8_t*>(k));
        ks.emplace_back(k, 20);
        key_block.push_back(off);
        fb.AddKey(Slice(ks.back()));
      }
      off += 700 + 211 * (b % 9);
      fb.StartBlock(off);  // TableBuilder::Flush
      ke.push_back(ks.size());
      eo.push_back(off);
    }
    Slice blk = fb.Finish();
    CHECK(fb.status() == DLSM_OK);
    std::string flat;
    std::vector<uint64_t> offs{0};
    for (auto& s : ks) {
      flat += s;
      offs.push_back(flat.size());
    }
    std::vector<uint8_t> want(64 * 1024, 0);
    int64_t wl = orc_filter_block_build(reinterpret_cast<const uint8_t*>(flat.data()), offs.data(), 0,
                                        ks.size(), ke.data(), eo.data(), static_cast<int>(ke.size()), 0,
                                        10, want.data(), want.size());
    CHECK(wl > 0 && static_cast<int64_t>(blk.size()) == wl);
    CHECK(std::memcmp(blk.data(), want.data(), wl) == 0);
    dlsm_adapter::FilterBlockReader rd(blk, ctx);
    for (size_t i = 0; i < ks.size(); i += 3)
      CHECK(rd.KeyMayMatch(key_block[i], Slice(ks[i])) ==
            (orc_filter_block_key_may_match(want.data(), wl, key_block[i],
                                            reinterpret_cast<const uint8_t*>(ks[i].data()), 20, 0) != 0));
  }
  // ---- hash_in_addkey: AddKey hashes on the host (block / AVX-512 forms),
  // Finish sends the hashes; variable-length keys with sign-extended tails,
  // runs of repeated keys, and 20-byte runs that straddle hash blocks; alone,
  // through a batcher, and with the hashes from 20-byte keys only ----
  {
    dlsm_batcher* bat = nullptr;
    CHECK(dlsm_batcher_create(0, 2, 0, 16, &bat) == DLSM_OK);
    for (int shape = 0; shape < 3; shape++) {
      for (int via_batcher = 0; via_batcher < 2; via_batcher++) {
        std::vector<char> slot(1 << 20, 0);
        dlsm_adapter::FilterSlot mr{slot.data(), slot.size()};
        dlsm_adapter::BuilderOptions opt;
        opt.hash_in_addkey = true;
        if (via_batcher) opt.batcher = bat;
        dlsm_adapter::FullFilterBlockBuilder b(&mr, 10, ctx, opt);
        std::string flat;
        std::vector<uint64_t> offs{0};
        uint32_t x = 777u + shape;
        const int n = shape == 0 ? 70001 : 9000;
        for (int i = 0; i < n; i++) {
          std::string k;
          if (shape == 0 || (shape == 2 && i % 300 < 250)) {  // 20-byte db_bench keys
            uint8_t kk[20];
            orc_dbbench_key(static_cast<uint64_t>(i), 20, kk);
            k.assign(reinterpret_cast<char*>(kk), 20);
          } else {  // 0..33 random bytes (>= 0x80 included: sign-extended tails)
            x = x * 1664525u + 1013904223u;
            const int len = static_cast<int>(x >> 27);
            for (int j = 0; j < len; j++) {
              x = x * 1664525u + 1013904223u;
              k.push_back(static_cast<char>(x >> 24));
            }
          }
          const int reps = (i % 11 == 0) ? 3 : 1;  // consecutive duplicates
          for (int r = 0; r < reps; r++) {
            b.AddKey(Slice(k));
            flat += k;
            offs.push_back(flat.size());
          }
        }
        b.Finish();
        CHECK(b.status() == DLSM_OK);
        std::vector<uint8_t> want(1 << 20, 0);
        const int64_t wl = orc_full_build(reinterpret_cast<const uint8_t*>(flat.data()), offs.data(), 0,
                                          offs.size() - 1, 10, want.data(), want.size());
        CHECK(wl > 0 && static_cast<int64_t>(b.result.size()) == wl);
        CHECK(std::memcmp(b.result.data(), want.data(), wl) == 0);
      }
    }
    dlsm_batcher_destroy(bat);
  }
  // ---- two live builders on ONE context: the second stages into a
  // private pinned buffer, both filters stay exact; keys over PCIe, then
  // hashes (the first streams them to the context's device buffer during
  // AddKey, the second hands them over in Finish) ----
  for (int hm = 0; hm < 2; hm++) {
    const int n1 = 40000, n2 = 70000;  // the second grows past the first's size
    std::vector<char> s1(256 * 1024, 0), s2(256 * 1024, 0);
    dlsm_adapter::FilterSlot m1{s1.data(), s1.size()}, m2{s2.data(), s2.size()};
    dlsm_adapter::BuilderOptions bo;
    bo.hash_in_addkey = hm == 1;
    dlsm_adapter::FullFilterBlockBuilder b1(&m1, 10, ctx, bo), b2(&m2, 10, ctx, bo);
    std::string f1, f2;
    std::vector<uint64_t> o1{0}, o2{0};
    for (int i = 0; i < n2; i++) {  // interleaved, as two tables' iterators would be
      uint8_t k[20];
      if (i < n1) {
        orc_dbbench_key(static_cast<uint64_t>(i) * 2, 20, k);
        b1.AddKey(Slice(reinterpret_cast<char*>(k), 20));
        f1.append(reinterpret_cast<char*>(k), 20);
        o1.push_back(f1.size());
      }
      orc_dbbench_key(static_cast<uint64_t>(i) * 2 + 1, 20, k);
      b2.AddKey(Slice(reinterpret_cast<char*>(k), 20));
      f2.append(reinterpret_cast<char*>(k), 20);
      o2.push_back(f2.size());
    }
    b1.Finish();
    b2.Finish();
    CHECK(b1.status() == DLSM_OK && b2.status() == DLSM_OK);
    std::vector<uint8_t> w1(256 * 1024, 0), w2(256 * 1024, 0);
    const int64_t l1 = orc_full_build(reinterpret_cast<const uint8_t*>(f1.data()), o1.data(), 0, n1, 10, w1.data(),
                                      w1.size());
    const int64_t l2 = orc_full_build(reinterpret_cast<const uint8_t*>(f2.data()), o2.data(), 0, n2, 10, w2.data(),
                                      w2.size());
    CHECK(static_cast<int64_t>(b1.result.size()) == l1 && std::memcmp(b1.result.data(), w1.data(), l1) == 0);
    CHECK(static_cast<int64_t>(b2.result.size()) == l2 && std::memcmp(b2.result.data(), w2.data(), l2) == 0);
  }
  // ---- Move_buffer outside the slot: refused unless its size is given and
  // holds the filter; the caller's BUILD_EXACT setting survives a Finish
  // over repeated keys ----
  {
    std::vector<char> slot(256 * 1024, 0), other(4096, 0);
    dlsm_adapter::FilterSlot mr{slot.data(), slot.size()};
    dlsm_adapter::FullFilterBlockBuilder b(&mr, 10, ctx);
    CHECK(dlsm_ctx_set_option(ctx, DLSM_OPT_BUILD_EXACT, 2) == DLSM_OK);
    auto add = [&](int n) {
      for (int i = 0; i < n; i++) {
        uint8_t k[20];
        orc_dbbench_key(static_cast<uint64_t>(i / 2), 20, k);  // every key twice
        b.AddKey(Slice(reinterpret_cast<char*>(k), 20));
      }
    };
    b.Move_buffer(other.data());  // no size: refused
    add(10000);
    b.Finish();
    CHECK(b.status() == DLSM_E_CAPACITY && b.result.size() == 0);
    b.Move_buffer(other.data(), other.size());  // 4 KiB < the 5,000-key filter's 6,341 bytes
    add(10000);
    b.Finish();
    // too small: the 69-byte match-everything filter, never a 0-byte one
    CHECK(b.status() == DLSM_E_CAPACITY && b.result.size() == 69 && !b.fell_back());
    for (int i = 0; i < 64; i++) CHECK(static_cast<uint8_t>(other[i]) == 0xff);
    CHECK(other[64] == 6 && other[65] == 1 && other[66] == 0 && other[67] == 0 && other[68] == 0);
    b.Move_buffer(other.data(), other.size());
    add(2000);  // 1,000 distinct keys: 1,349 bytes
    b.Finish();
    CHECK(b.status() == DLSM_OK && b.result.size() == 1349 && b.result.data() == other.data());
    uint64_t ex = 99;
    CHECK(dlsm_ctx_get_option(ctx, DLSM_OPT_BUILD_EXACT, &ex) == DLSM_OK && ex == 2);
    CHECK(dlsm_ctx_set_option(ctx, DLSM_OPT_BUILD_EXACT, 0) == DLSM_OK);
  }
  // no call of this test fell back to the host: the GPU served all of them
  uint64_t fb_ctx = 1, fb_all = 1;
  CHECK(dlsm_fallback_stats(ctx, &fb_ctx, &fb_all) == DLSM_OK && fb_ctx == 0 && fb_all == 0);
  dlsm_ctx_destroy(ctx);
  std::printf("OK adapter\n");
  return 0;
}
