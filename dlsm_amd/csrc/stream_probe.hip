// dlsm_amd/csrc/stream_probe.hip -- the box's own HBM streaming ceilings,
// measured in the same run as the bench (bench.py stream_ceilings): plain
// 16-byte-per-lane read-only and copy kernels, the achievable rates the
// Bloom passes are compared against beside the 8 TB/s spec peak.  Not on the
// filter path.
//
// Shapes (variant bits): bit 0 -- non-temporal loads / stores; bit 1 -- each
// workgroup streams one contiguous range (else a grid-stride loop, every wave
// instruction 1 KiB contiguous); UNROLL = 8 16-byte loads in flight per lane.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/dlsm_bloom.h"

namespace {
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, const u32x4& v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

constexpr int kU = 8;
constexpr int kNT = 512;

// [first, end) of this thread's walk, and its step: grid-stride, or one
// contiguous range per workgroup walked block-wide.
template <bool CHUNKED>
__device__ __forceinline__ void range(uint64_t n16, uint64_t& i, uint64_t& end, uint64_t& step) {
  if constexpr (CHUNKED) {
    const uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = per * blockIdx.x;
    i = b0 + threadIdx.x;
    end = b0 + per < n16 ? b0 + per : n16;
    step = kNT;
  } else {
    i = static_cast<uint64_t>(blockIdx.x) * kNT + threadIdx.x;
    end = n16;
    step = static_cast<uint64_t>(gridDim.x) * kNT;
  }
}

template <bool NT, bool CHUNKED>
__global__ __launch_bounds__(kNT) void read_kernel(const u32x4* __restrict__ src, uint64_t n16,
                                                   uint32_t* __restrict__ sink) {
  uint64_t i, end, step;
  range<CHUNKED>(n16, i, end, step);
  uint32_t acc = 0;
  for (; i + (kU - 1) * step < end; i += kU * step) {
    u32x4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) v[u] = ld<NT>(src + i + u * step);
#pragma unroll
    for (int u = 0; u < kU; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < end; i += step) acc ^= ld<NT>(src + i).x;
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;  // keeps the loads; never true for the bench's zeros
}

template <bool NT, bool CHUNKED>
__global__ __launch_bounds__(kNT) void copy_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                   uint64_t n16) {
  uint64_t i, end, step;
  range<CHUNKED>(n16, i, end, step);
  for (; i + (kU - 1) * step < end; i += kU * step) {
    u32x4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) v[u] = ld<NT>(src + i + u * step);
#pragma unroll
    for (int u = 0; u < kU; u++) st<NT>(dst + i + u * step, v[u]);
  }
  for (; i < end; i += step) st<NT>(dst + i, ld<NT>(src + i));
}

// The probe partition's byte shape: 20 B read and 6 B written per key, as a
// read stream and a write stream of 16-byte units in the ratio 10 : 3.
template <bool NT, bool CHUNKED>
__global__ __launch_bounds__(kNT) void part_shape_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                         uint64_t n16) {
  uint64_t i, end, step;
  range<CHUNKED>(n16, i, end, step);
  // this thread's write position: the same walk over a range 3/10 as long
  uint64_t w = CHUNKED ? (i - threadIdx.x) / 10 * 3 + threadIdx.x : i;
  for (; i + 9 * step < end; i += 10 * step, w += 3 * step) {
    u32x4 v[10];
#pragma unroll
    for (int u = 0; u < 10; u++) v[u] = ld<NT>(src + i + u * step);
    const u32x4 a = v[0] ^ v[1] ^ v[2], b = v[3] ^ v[4] ^ v[5], c = v[6] ^ v[7] ^ v[8] ^ v[9];
    st<NT>(dst + w, a);
    st<NT>(dst + w + step, b);
    st<NT>(dst + w + 2 * step, c);
  }
}

template <bool NT, bool CHUNKED>
hipError_t launch(int kind, const void* src, void* dst, uint64_t n16, unsigned blocks, hipStream_t s) {
  if (kind == 2)
    part_shape_kernel<NT, CHUNKED><<<blocks, kNT, 0, s>>>(static_cast<const u32x4*>(src), static_cast<u32x4*>(dst),
                                                          n16);
  else if (kind == 0)
    read_kernel<NT, CHUNKED><<<blocks, kNT, 0, s>>>(static_cast<const u32x4*>(src), n16,
                                                     static_cast<uint32_t*>(dst));
  else
    copy_kernel<NT, CHUNKED><<<blocks, kNT, 0, s>>>(static_cast<const u32x4*>(src), static_cast<u32x4*>(dst),
                                                     n16);
  return hipGetLastError();
}
}  // namespace

extern "C" int dlsm_stream_kernel(void* hip_stream, int kind, int variant, const void* src, void* dst,
                                  uint64_t bytes, uint32_t blocks) {
  if (kind < 0 || kind > 2 || variant < 0 || variant > 3 || !src || !dst || blocks == 0 || (bytes & 15u))
    return DLSM_E_ARG;
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) return DLSM_E_ARG;
  const uint64_t n16 = bytes / 16;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  hipError_t e;
  switch (variant) {
    case 0: e = launch<false, false>(kind, src, dst, n16, blocks, s); break;
    case 1: e = launch<true, false>(kind, src, dst, n16, blocks, s); break;
    case 2: e = launch<false, true>(kind, src, dst, n16, blocks, s); break;
    default: e = launch<true, true>(kind, src, dst, n16, blocks, s); break;
  }
  return e == hipSuccess ? DLSM_OK : DLSM_E_DEVICE;
}
