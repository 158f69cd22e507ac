// Diagnostic only: the cost of key staging in each kind of host memory --
// AddKey's 20-byte appends (CPU writes) and Finish's H2D copy of the staged
// table (DMA).  hipHostMalloc default / non-coherent / write-combined, and
// malloc'd pages page-locked with hipHostRegister, against plain pageable
// memory.  Prints one JSON line.  Build and run on a GPU box:
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 tests/diag/host_staging.hip -o host_staging && ./host_staging
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using Clock = std::chrono::steady_clock;

int main() {
  const size_t n = 153846, key = 20, bytes = n * key, reps = 20;
  std::vector<uint8_t> src(bytes);
  for (size_t i = 0; i < bytes; i++) src[i] = static_cast<uint8_t>(i * 131u + 7u);
  void* dev = nullptr;
  if (hipMalloc(&dev, bytes) != hipSuccess) return 1;
  hipStream_t s;
  (void)hipStreamCreate(&s);
  struct Kind {
    const char* name;
    int how;  // 0 malloc, 1..3 hipHostMalloc flags, 4 malloc + hipHostRegister
    unsigned flags;
  } kinds[] = {{"pageable malloc", 0, 0},
               {"hipHostMalloc default", 1, hipHostMallocDefault},
               {"hipHostMalloc non-coherent", 1, hipHostMallocNonCoherent},
               {"hipHostMalloc write-combined", 1, hipHostMallocWriteCombined},
               {"malloc + hipHostRegister", 4, 0}};
  std::string out = "{\"keys\": 153846, \"key_bytes\": 20, \"kinds\": [";
  bool first = true;
  for (const Kind& k : kinds) {
    void* p = nullptr;
    if (k.how == 0 || k.how == 4) {
      p = std::aligned_alloc(4096, (bytes + 4095) / 4096 * 4096);
      if (k.how == 4 && hipHostRegister(p, (bytes + 4095) / 4096 * 4096, hipHostRegisterDefault) != hipSuccess) {
        std::free(p);
        continue;
      }
    } else if (hipHostMalloc(&p, bytes, k.flags) != hipSuccess) {
      continue;
    }
    uint8_t* q = static_cast<uint8_t*>(p);
    std::memset(q, 0, bytes);
    // AddKey-shaped writes: one 20-byte memcpy per key
    double wbest = 1e30, cbest = 1e30, rbest = 1e30;
    for (size_t r = 0; r < reps; r++) {
      const auto t0 = Clock::now();
      for (size_t i = 0; i < n; i++) std::memcpy(q + i * key, src.data() + i * key, key);
      const auto t1 = Clock::now();
      wbest = std::min(wbest, std::chrono::duration<double, std::nano>(t1 - t0).count() / n);
      // reading the previous key back (the duplicate check of the r2 adapter)
      uint32_t acc = 0;
      const auto t2 = Clock::now();
      for (size_t i = 0; i < n; i++) acc += q[i * key + (i & 15)];
      const auto t3 = Clock::now();
      if (acc == 0xdeadbeef) std::printf("x");
      rbest = std::min(rbest, std::chrono::duration<double, std::nano>(t3 - t2).count() / n);
      const auto t4 = Clock::now();
      (void)hipMemcpyAsync(dev, q, bytes, hipMemcpyHostToDevice, s);
      (void)hipStreamSynchronize(s);
      const auto t5 = Clock::now();
      cbest = std::min(cbest, std::chrono::duration<double, std::micro>(t5 - t4).count());
    }
    char buf[400];
    std::snprintf(buf, sizeof(buf),
                  "%s{\"kind\": \"%s\", \"addkey_write_ns_per_key\": %.2f, \"read_ns_per_key\": %.2f, "
                  "\"h2d_us\": %.1f, \"h2d_GBs\": %.1f}",
                  first ? "" : ", ", k.name, wbest, rbest, cbest, bytes / (cbest * 1e3));
    out += buf;
    first = false;
    if (k.how == 0) std::free(p);
    else if (k.how == 4) {
      (void)hipHostUnregister(p);
      std::free(p);
    } else {
      (void)hipHostFree(p);
    }
  }
  out += "]}";
  std::printf("%s\n", out.c_str());
  return 0;
}
