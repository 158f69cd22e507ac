// Diagnostic only: the HBM streaming ceilings of a box, for the probe
// partition's "at the streaming ceiling" claim.  Three shapes,
// each a persistent grid-stride loop of 16-byte accesses, UNROLL loads in
// flight per lane:
//   kind 0  read-only (XOR-folded, one dword written per thread at the end)
//   kind 1  copy (read 16 B, write 16 B)
//   kind 2  the partition's shape: read 20 B per key (five 16-B loads per
//           four keys' 80 B), write 4 B + 2 B per key (non-temporal)
// tests/diag/run_stream_ceiling.py drives it.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL>
__global__ __launch_bounds__(512) void read_kernel(const uint4* __restrict__ src, uint64_t n16, uint32_t* out) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n16; i += stride) acc ^= src[i].x;
  out[static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x] = acc;
}

template <int UNROLL>
__global__ __launch_bounds__(512) void copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                   uint64_t n16) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
    uint4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) dst[i + u * stride] = v[u];
  }
  for (; i < n16; i += stride) dst[i] = src[i];
}

// four keys (80 B) per lane-step: five 16-B loads; write 16 B of "entries"
// and 8 B of "positions" per four keys (non-temporal)
template <int UNROLL>
__global__ __launch_bounds__(512) void part_kernel(const uint4* __restrict__ keys, uint4* __restrict__ ent,
                                                   uint2* __restrict__ pos, uint64_t n4) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n4; i += UNROLL * stride) {
    uint4 v[UNROLL][5];
#pragma unroll
    for (int u = 0; u < UNROLL; u++)
#pragma unroll
      for (int j = 0; j < 5; j++) v[u][j] = keys[(i + u * stride) * 5 + j];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      uint32_t h[4];
      h[0] = v[u][0].x ^ v[u][0].y ^ v[u][0].z ^ v[u][0].w ^ v[u][1].x;
      h[1] = v[u][1].y ^ v[u][1].z ^ v[u][1].w ^ v[u][2].x ^ v[u][2].y;
      h[2] = v[u][2].z ^ v[u][2].w ^ v[u][3].x ^ v[u][3].y ^ v[u][3].z;
      h[3] = v[u][3].w ^ v[u][4].x ^ v[u][4].y ^ v[u][4].z ^ v[u][4].w;
      u32x4 e = {h[0], h[1], h[2], h[3]};
      __builtin_nontemporal_store(e, reinterpret_cast<u32x4*>(ent + i + u * stride));
      pos[i + u * stride] = make_uint2((h[0] & 0xffff) | (h[1] << 16), (h[2] & 0xffff) | (h[3] << 16));
    }
  }
}
}  // namespace

extern "C" int stream_ceiling_launch(int kind, const void* src, void* dst, void* dst2, uint64_t bytes, int blocks,
                                     int unroll) {
  const dim3 g(blocks), b(512);
  if (kind == 0) {
    const uint64_t n16 = bytes / 16;
    auto* o = static_cast<uint32_t*>(dst);
    if (unroll == 4) read_kernel<4><<<g, b>>>(static_cast<const uint4*>(src), n16, o);
    else read_kernel<8><<<g, b>>>(static_cast<const uint4*>(src), n16, o);
  } else if (kind == 1) {
    const uint64_t n16 = bytes / 16;
    if (unroll == 4) copy_kernel<4><<<g, b>>>(static_cast<const uint4*>(src), static_cast<uint4*>(dst), n16);
    else copy_kernel<8><<<g, b>>>(static_cast<const uint4*>(src), static_cast<uint4*>(dst), n16);
  } else {
    const uint64_t n4 = bytes / 80;  // groups of four 20-byte keys
    if (unroll == 2)
      part_kernel<2><<<g, b>>>(static_cast<const uint4*>(src), static_cast<uint4*>(dst), static_cast<uint2*>(dst2), n4);
    else
      part_kernel<1><<<g, b>>>(static_cast<const uint4*>(src), static_cast<uint4*>(dst), static_cast<uint2*>(dst2), n4);
  }
  return static_cast<int>(hipGetLastError());
}
