// Diagnostic (run by hand on a GPU box; results under profiles/): the random
// byte gather of the probe slice pass (probe_slice_kernel: 6 one-byte probes
// per entry, each in a random 512-byte stacked line of a 125 KiB LDS slice),
// in isolation, by LDS instruction:
//   u8      ds_read_u8 of the probed byte (the product's form)
//   b32     ds_read_b32 of its aligned dword + a shift
//   b64     ds_read_b64 of its aligned 8 bytes + a shift
//   nocf    ds_read_u8 with every lane of a 32-lane group on its own bank
//           (the conflict-free floor of the same instruction count)
//   pred3   ds_read_u8, probes 3..5 only while the AND of probes 0..2 is not 0
//           (one dependent round instead of none; masked lanes issue no read)
//   valu    the address and AND arithmetic without LDS reads
// One 1,024-thread workgroup per CU, ITER windows of 4 entries per lane; the
// positions come from a per-lane hash stream like the entries' (x += delta).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tests/diag/lds_gather.hip -o /tmp/ldsg && /tmp/ldsg
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int NT = 1024;
constexpr int LINES = 245;  // the bench slice: 245 stacked lines of 512 bytes
constexpr int ITER = 4000;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  return x ^ (x >> 16);
}

template <int V>
__global__ __launch_bounds__(NT) void gather(uint32_t seed, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t sl[LINES * 512];
  for (int i = threadIdx.x; i < LINES * 512 / 4; i += NT)
    reinterpret_cast<uint32_t*>(sl)[i] = mix(i * 2654435761u + seed) | 0x01010101u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t st = mix(seed ^ (blockIdx.x * NT + threadIdx.x));
  uint32_t sink = 0;
  for (int it = 0; it < ITER; it++) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      st = st * 1664525u + 1013904223u;
      uint32_t x = mix(st);
      const uint32_t base = (x >> 24) % LINES * 512u;
      const uint32_t delta = x >> 17;
      uint32_t acc = 0xffu;
      if constexpr (V == 5) {  // valu only
#pragma unroll
        for (int q = 0; q < 6; q++) {
          acc &= (base | (x & 511u)) | 0xf0u;
          x += delta;
        }
      } else if constexpr (V == 4) {  // probes 3..5 predicated on probes 0..2
        uint32_t a3 = 0xffu;
#pragma unroll
        for (int q = 0; q < 3; q++) {
          a3 &= sl[base | (x & 511u)];
          x += delta;
        }
        if (a3) {
#pragma unroll
          for (int q = 3; q < 6; q++) {
            a3 &= sl[base | (x & 511u)];
            x += delta;
          }
        }
        acc = a3;
      } else {
#pragma unroll
        for (int q = 0; q < 6; q++) {
          uint32_t p = x & 511u;
          if constexpr (V == 3) p = (p & ~(31u << 2)) | ((lane & 31u) << 2);  // own bank per lane
          const uint32_t a = base | p;
          if constexpr (V == 0 || V == 3) {
            acc &= sl[a];
          } else if constexpr (V == 1) {
            acc &= reinterpret_cast<const uint32_t*>(sl)[a >> 2] >> ((a & 3u) * 8u);
          } else {
            acc &= static_cast<uint32_t>(reinterpret_cast<const uint64_t*>(sl)[a >> 3] >> ((a & 7u) * 8u));
          }
          x += delta;
        }
      }
      sink += acc & 0xffu;
    }
  }
  if (sink == 0x12345678u) out[blockIdx.x] = sink;  // keeps the reads
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* out = nullptr;
  (void)hipMalloc(&out, 4096 * sizeof(uint32_t));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[6] = {"u8", "b32", "b64", "nocf", "pred3", "valu"};
  const double probes = static_cast<double>(cus) * NT * ITER * 4 * 6;  // pred3 issues fewer
  for (int round = 0; round < 2; round++) {
    for (int v = 0; v < 6; v++) {
      auto launch = [&] {
        switch (v) {
          case 0: gather<0><<<cus, NT>>>(round + 1, out); break;
          case 1: gather<1><<<cus, NT>>>(round + 1, out); break;
          case 2: gather<2><<<cus, NT>>>(round + 1, out); break;
          case 3: gather<3><<<cus, NT>>>(round + 1, out); break;
          case 4: gather<4><<<cus, NT>>>(round + 1, out); break;
          default: gather<5><<<cus, NT>>>(round + 1, out); break;
        }
      };
      launch();
      (void)hipEventRecord(e0);
      for (int r = 0; r < 5; r++) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double s = ms / 5 / 1e3;
      // the product's slice pass does 600 M such probes (100 M keys x 6)
      std::printf("{\"variant\": \"%s\", \"cus\": %d, \"ms\": %.3f, \"gprobes_s\": %.1f, "
                  "\"us_per_600M_probes\": %.1f}\n",
                  names[v], cus, s * 1e3, probes / s / 1e9, 600e6 / (probes / s) * 1e6);
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
