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
//   u8io    u8 with the slice pass's memory side: each lane loads its window
//           of 4 entries as one 16-byte unit from HBM and stores their 4
//           answer bytes as one dword (the product's 4 B in, 1 B out per key)
//   io      the same loads and stores and arithmetic, no LDS reads
// One 1,024-thread workgroup per CU, ITER windows of 4 entries per lane
// (~100 M entries per launch, the bench's lookup count); the positions come
// from a per-lane hash stream like the entries' (x += delta), or from the
// loaded entries for u8io / io.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tests/diag/lds_gather.hip -o /tmp/ldsg && /tmp/ldsg
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int NT = 1024;
constexpr int LINES = 245;  // the bench slice: 245 stacked lines of 512 bytes
constexpr int ITER = 96;  // 256 CUs x 1,024 lanes x 96 x 4 = 100.7 M entries

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  return x ^ (x >> 16);
}

template <int V>
__global__ __launch_bounds__(NT) void gather(uint32_t seed, uint32_t* out, const uint4* ent, uint32_t* ans) {
  __shared__ __attribute__((aligned(16))) uint8_t sl[LINES * 512];
  for (int i = threadIdx.x; i < LINES * 512 / 4; i += NT)
    reinterpret_cast<uint32_t*>(sl)[i] = mix(i * 2654435761u + seed) | 0x01010101u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t st = mix(seed ^ (blockIdx.x * NT + threadIdx.x));
  uint32_t sink = 0;
  const uint64_t gt = static_cast<uint64_t>(blockIdx.x) * NT + threadIdx.x;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * NT;
  for (int it = 0; it < ITER; it++) {
    uint4 e = make_uint4(0, 0, 0, 0);
    if constexpr (V >= 6) e = ent[it * stride + gt];
    const uint32_t e4[4] = {e.x, e.y, e.z, e.w};
    uint32_t a4 = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint32_t x;
      if constexpr (V >= 6) {
        x = e4[j];
      } else {
        st = st * 1664525u + 1013904223u;
        x = mix(st);
      }
      const uint32_t base = (x >> 24) % LINES * 512u;
      const uint32_t delta = x >> 17;
      uint32_t acc = 0xffu;
      if constexpr (V == 5 || V == 7) {  // valu only
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
          if constexpr (V == 0 || V == 3 || V == 6) {
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
      a4 |= (acc & 0xffu) << (8 * j);
    }
    if constexpr (V >= 6) ans[it * stride + gt] = a4;
  }
  if (sink == 0x12345678u) out[blockIdx.x] = sink;  // keeps the reads
}

__global__ void fill(uint32_t* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x)
    p[i] = mix(static_cast<uint32_t>(i) * 0x9E3779B9u + 7u);
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* out = nullptr;
  (void)hipMalloc(&out, 4096 * sizeof(uint32_t));
  const uint64_t n_ent = static_cast<uint64_t>(cus) * NT * ITER * 4;
  uint32_t *ent = nullptr, *ans = nullptr;
  (void)hipMalloc(&ent, n_ent * 4);
  (void)hipMalloc(&ans, n_ent);
  fill<<<4096, 256>>>(ent, n_ent);
  const uint4* ent4 = reinterpret_cast<const uint4*>(ent);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[8] = {"u8", "b32", "b64", "nocf", "pred3", "valu", "u8io", "io"};
  const double probes = static_cast<double>(cus) * NT * ITER * 4 * 6;  // pred3 issues fewer
  for (int round = 0; round < 2; round++) {
    for (int v = 0; v < 8; v++) {
      auto launch = [&] {
        switch (v) {
          case 0: gather<0><<<cus, NT>>>(round + 1, out, ent4, ans); break;
          case 1: gather<1><<<cus, NT>>>(round + 1, out, ent4, ans); break;
          case 2: gather<2><<<cus, NT>>>(round + 1, out, ent4, ans); break;
          case 3: gather<3><<<cus, NT>>>(round + 1, out, ent4, ans); break;
          case 4: gather<4><<<cus, NT>>>(round + 1, out, ent4, ans); break;
          case 5: gather<5><<<cus, NT>>>(round + 1, out, ent4, ans); break;
          case 6: gather<6><<<cus, NT>>>(round + 1, out, ent4, ans); break;
          default: gather<7><<<cus, NT>>>(round + 1, out, ent4, ans); break;
        }
      };
      launch();
      (void)hipEventRecord(e0);
      for (int r = 0; r < 20; r++) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double s = ms / 20 / 1e3;
      // the product's slice pass does 600 M such probes (100 M keys x 6)
      std::printf("{\"variant\": \"%s\", \"cus\": %d, \"us\": %.1f, \"gprobes_s\": %.1f, "
                  "\"us_per_600M_probes\": %.1f, \"io_GBs\": %.0f}\n",
                  names[v], cus, s * 1e6, probes / s / 1e9, 600e6 / (probes / s) * 1e6,
                  v >= 6 ? n_ent * 5.0 / s / 1e9 : 0.0);
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
