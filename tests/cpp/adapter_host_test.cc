// Host-only checks of the C++ adapter (no GPU, no context): where Finish may
// write after Move_buffer (full_filter_block.cc:144-146), and the staging
// buffer's claim rules.  Built and run by tests/test_gpu_adapter.py on CPU.
#include <cstdio>
#include <vector>

#include "dlsm_bloom_adapter.hpp"

#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      return 1;                                               \
    }                                                         \
  } while (0)

int main() {
  std::vector<char> slot(256 * 1024), other(4096);
  dlsm_adapter::FilterSlot mr{slot.data(), slot.size()};
  dlsm_adapter::FullFilterBlockBuilder b(&mr, 10, nullptr);
  CHECK(b.output_capacity() == slot.size());  // a fresh builder writes at the slot's start
  b.Move_buffer(slot.data() + 1000);           // inside the slot: the rest of it
  CHECK(b.output_capacity() == slot.size() - 1000);
  b.Move_buffer(slot.data());                  // what every reference caller does
  CHECK(b.output_capacity() == slot.size());
  b.Move_buffer(other.data());                 // outside, size unknown: nothing may be written
  CHECK(b.output_capacity() == 0);
  b.Move_buffer(other.data(), other.size());   // outside with its size
  CHECK(b.output_capacity() == other.size());
  b.Reset();                                   // back to the slot (full_filter_block.cc:141-143)
  CHECK(b.output_capacity() == slot.size());
  // the header's inline BloomHash (AddKey's host hashing) == the library's,
  // lengths 0..70 with bytes >= 0x80 in every tail position (sign extension)
  {
    std::vector<char> k(70);
    uint32_t x = 12345u;
    for (int rep = 0; rep < 40; rep++) {
      for (auto& c : k) {
        x = x * 1664525u + 1013904223u;
        c = static_cast<char>(x >> 24);
      }
      for (size_t n = 0; n <= k.size(); n++)
        CHECK(dlsm_adapter::BloomHash(k.data(), n) == dlsm_bloom_hash(k.data(), n));
    }
    CHECK(dlsm_adapter::BloomHash("\xc3\x97", 2) == 0x0f2ba540u);  // the reference code's value
    // the 4- and 16-key block forms AddKey uses for 20-byte keys
    std::vector<char> b(320 * 50);
    for (auto& c : b) {
      x = x * 1664525u + 1013904223u;
      c = static_cast<char>(x >> 24);
    }
    for (size_t o = 0; o + 320 <= b.size(); o += 320) {
      uint32_t h4[4], h16[16];
      dlsm_adapter::BloomHash20x4(b.data() + o, h4);
      dlsm_adapter::BloomHash20x16(b.data() + o, h16);
      for (int i = 0; i < 16; i++) CHECK(h16[i] == dlsm_bloom_hash(b.data() + o + 20 * i, 20));
      for (int i = 0; i < 4; i++) CHECK(h4[i] == h16[i]);
    }
  }
  // the staging-buffer claim needs a context
  CHECK(dlsm_ctx_host_buffer_claim(nullptr, &b) == DLSM_E_ARG);
  CHECK(dlsm_ctx_host_buffer_release(nullptr, &b) == DLSM_E_ARG);
  std::printf("OK adapter host\n");
  return 0;
}
