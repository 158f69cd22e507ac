// Diagnostic only (never part of the library): the probe slice kernel exactly
// as it stood before commit 1c7c4c6 ("Fix sliced-probe corruption"), built
// in several variants -- that commit's __launch_bounds__(1024, 8) (forces <= 64 VGPRs,
// the compiler spills one VGPR) and with __launch_bounds__(1024) -- so the
// corruption can be reproduced in isolation and its cause pinned
// (tests/diag/run_old_slice.py).
//
// Layout of that era: 4,096-key chunks, each chunk region holds the chunk's
// raw 32-bit hashes grouped by slice of 128 stacked lines; tab = chunk-major
// rows of S+1 u16 bucket starts; stacked = per line 64 uint64 words, byte f
// of word w = byte w of filter f's line.  smask[i] = answer of entries[i].
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
constexpr int kChunk = 4096;
constexpr int kNT = 1024;

__device__ __forceinline__ uint32_t fastmod(uint32_t h, uint32_t d, uint32_t magic) {
  const uint32_t q = __umulhi(h, magic);
  const uint32_t r = h - q * d;
  return r >= d ? r - d : r;
}
__device__ __forceinline__ uint32_t bloom_delta(uint32_t h) { return (h >> 17) | (h << 15); }

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

__device__ __forceinline__ void seg_locate(uint32_t excl, uint32_t off, uint32_t T, uint32_t b0,
                                           uint32_t& sc, uint32_t& li, uint32_t& st, uint32_t& of) {
  while (sc + 1 < 64 && static_cast<uint32_t>(__builtin_amdgcn_readlane(excl, sc + 1)) <= b0) sc++;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t e = min(b0 + lane, T - 1u);
  const uint32_t last = min(b0 + 63u, T - 1u);
  li = sc;
  st = static_cast<uint32_t>(__builtin_amdgcn_readlane(excl, sc));
  of = static_cast<uint32_t>(__builtin_amdgcn_readlane(off, sc));
  for (uint32_t j = sc + 1; j < 64; j++) {
    const uint32_t bj = static_cast<uint32_t>(__builtin_amdgcn_readlane(excl, j));
    if (bj > last) break;
    const uint32_t oj = static_cast<uint32_t>(__builtin_amdgcn_readlane(off, j));
    if (e >= bj) {
      li = j;
      st = bj;
      of = oj;
    }
  }
}

// MINW: the launch bound's waves per SIMD; kU: windows per lane (8 then);
// PADKB: extra LDS per workgroup (88 KiB keeps one workgroup per CU).
template <int MINW, int kU, int PADKB>
__global__ __launch_bounds__(kNT, MINW) void old_slice_kernel(
    const uint64_t* __restrict__ stacked, uint32_t L, uint32_t magic, uint32_t S, uint32_t nC,
    const uint32_t* __restrict__ entries, const uint16_t* __restrict__ tab, uint8_t* __restrict__ smask,
    int parts) {
  constexpr int LGR = 7, K = 6;
  constexpr uint32_t R = 1u << LGR;
  constexpr int NW = kNT / 64;
  __shared__ __attribute__((aligned(16))) uint64_t sl[R * 64 + PADKB * 128];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t s = blockIdx.x % S;
  const uint32_t p = blockIdx.x / S;
  const uint32_t lo_line = s << LGR;
  const uint32_t nl = min(R, L - lo_line);
  {
    const uint4* src = reinterpret_cast<const uint4*>(stacked + static_cast<uint64_t>(lo_line) * 64u);
    uint4* dst = reinterpret_cast<uint4*>(sl);
    const uint32_t nw = nl * 32u;
    uint4 t0 = src[min(static_cast<uint32_t>(0 * kNT + tid), nw - 1u)];
    uint4 t1 = src[min(static_cast<uint32_t>(1 * kNT + tid), nw - 1u)];
    uint4 t2 = src[min(static_cast<uint32_t>(2 * kNT + tid), nw - 1u)];
    uint4 t3 = src[min(static_cast<uint32_t>(3 * kNT + tid), nw - 1u)];
    if (0 * kNT + tid < nw) dst[0 * kNT + tid] = t0;
    if (1 * kNT + tid < nw) dst[1 * kNT + tid] = t1;
    if (2 * kNT + tid < nw) dst[2 * kNT + tid] = t2;
    if (3 * kNT + tid < nw) dst[3 * kNT + tid] = t3;
  }
  const uint32_t c_lo = static_cast<uint32_t>(static_cast<uint64_t>(p) * nC / parts);
  const uint32_t c_hi = static_cast<uint32_t>(static_cast<uint64_t>(p + 1) * nC / parts);
  const uint16_t* tb = tab + s;
  __syncthreads();
  for (uint32_t g = c_lo + wv * 64u; g < c_hi; g += NW * 64u) {
    const uint32_t c = g + lane;
    const uint16_t* r = tb + static_cast<uint64_t>(c) * (S + 1);
    const uint32_t o0 = c < c_hi ? r[0] : 0u;
    const uint32_t cnt = c < c_hi ? r[1] - o0 : 0u;
    const uint32_t incl = wave_incl_scan(cnt);
    const uint32_t excl = incl - cnt;
    const uint32_t T = __shfl(incl, 63, 64);
    uint32_t sc = 0;
    for (uint32_t e0 = 0; e0 < T; e0 += 64u * kU) {
      uint32_t hv[kU];
      uint64_t idx[kU];
      bool ok[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t b0 = e0 + u * 64u;
        ok[u] = b0 + lane < T;
        uint32_t li = 0, st = 0, of = 0;
        if (b0 < T) seg_locate(excl, o0, T, b0, sc, li, st, of);
        const uint32_t ec = min(b0 + lane, T - 1u);
        idx[u] = static_cast<uint64_t>(g + li) * kChunk + of + (ec - st);
        hv[u] = entries[idx[u]];
      }
#pragma unroll
      for (int u = 0; u < kU; u++) {
        if (!ok[u]) continue;
        uint32_t x = hv[u];
        const uint64_t* ln = sl + (fastmod(x, L, magic) - lo_line) * 64u;
        const uint32_t delta = bloom_delta(x);
        uint64_t acc = 0x0101010101010101ull;
        uint64_t v[K];
        uint32_t sh[K];
#pragma unroll
        for (int q = 0; q < K; q++) {
          const uint32_t bp = x & 511u;
          v[q] = ln[bp >> 3];
          sh[q] = bp & 7u;
          x += delta;
        }
#pragma unroll
        for (int q = 0; q < K; q++) acc &= v[q] >> sh[q];
        acc &= 0x0101010101010101ull;
        smask[idx[u]] = static_cast<uint8_t>((acc * 0x0102040810204080ull) >> 56);
      }
    }
  }
}
}  // namespace

// variants: 0 = the pre-fix kernel, __launch_bounds__(1024, 8), 8 windows
// (one VGPR spilled, two workgroups per CU); 1 = __launch_bounds__(1024)
// (65 VGPRs, no spill, one per CU); 2 = variant 0 with 24 KiB of extra LDS
// (spill kept, one workgroup per CU); 3 = (1024, 8) with 6 windows (no
// spill, two per CU).
extern "C" int old_slice_launch(const void* stacked, uint32_t L, uint32_t S, uint32_t nC,
                                const uint32_t* entries, const uint16_t* tab, uint8_t* smask, int parts,
                                int variant) {
  const uint32_t magic = 0xffffffffu / L;
  const dim3 grid(S * parts);
  const uint64_t* st = static_cast<const uint64_t*>(stacked);
#define OLD_SLICE(MW, UU, PK) \
  old_slice_kernel<MW, UU, PK><<<grid, kNT>>>(st, L, magic, S, nC, entries, tab, smask, parts)
  switch (variant) {
    case 0: OLD_SLICE(8, 8, 0); break;
    case 1: OLD_SLICE(1, 8, 0); break;
    case 2: OLD_SLICE(8, 8, 24); break;
    case 3: OLD_SLICE(8, 6, 0); break;
    default: return -3;
  }
#undef OLD_SLICE
  if (hipGetLastError() != hipSuccess) return -1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
