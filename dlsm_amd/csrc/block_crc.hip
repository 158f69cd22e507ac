// dlsm_amd/csrc/block_crc.hip -- crc32c (Castagnoli) on gfx950 for the
// filter-block trailer.
//
// FinishFilterBlock (table/table_builder_computeside.cc:418-428) appends
//   [type = kNoCompression (0)][Fixed32(crc32c::Mask(crc32c::Value(filter || type)))]
// to the filter before FlushFilter RDMA-writes it; ReadFilterBlock
// (table/format.cc:398-408) re-computes the same crc.  util/crc32c.h:17-37.
//
// Parallel form.  With r(D) the "raw" CRC (register starts at 0, no final
// inversion), r is GF(2)-linear and ignores leading zero bytes:
//   r(A||B) = r(A) * x^(8|B|)  xor  r(B)   (mod P),   r(0^k || D) = r(D),
// and the standard value is Value(D) = ~(0xffffffff * x^(8|D|) xor r(D)).
// So a stream is front-padded with zeros to whole 64 KiB parts; each thread
// takes 16 bytes (one coalesced 16-byte load), the wave and the workgroup
// fold pairs of equal-length neighbours with one constant x^(8*16*2^k) per
// level, and a second kernel folds the parts of each stream.
#include <hip/hip_runtime.h>

#include "bloom_internal.h"

namespace dlsm {
namespace {

constexpr uint32_t kCrcPoly = 0x82f63b78u;  // reflected Castagnoli polynomial
constexpr int kCrcBlock = 1024;             // threads per workgroup
constexpr uint32_t kCrcSub = kCrcBlock * 16u;         // 16 KiB per workgroup pass
constexpr uint32_t kCrcSubs = 4;                      // passes per part
constexpr uint64_t kCrcPart = kCrcSub * kCrcSubs;     // 64 KiB per workgroup

// a(x) * b(x) mod P in the reflected representation (bit 31 = x^0).
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    if (a & (0x80000000u >> i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ kCrcPoly : (b >> 1);
  }
  return p;
}

// x^(8n) mod P from the table xpow[k] = x^(2^k) mod P.
__device__ __forceinline__ uint32_t x8n(uint64_t n, const uint32_t* xpow) {
  uint32_t r = 0x80000000u;  // x^0
  n <<= 3;
  for (int k = 0; n; k++, n >>= 1)
    if (n & 1u) r = multmodp(r, xpow[k]);
  return r;
}

// Raw CRC of one little-endian word appended to register r (slice-by-4).
__device__ __forceinline__ uint32_t raw_word(uint32_t r, uint32_t w, const uint32_t* T) {
  r ^= w;
  return T[768 + (r & 0xffu)] ^ T[512 + ((r >> 8) & 0xffu)] ^ T[256 + ((r >> 16) & 0xffu)] ^
         T[r >> 24];
}

__device__ void build_tables(uint32_t* T) {
  // T[0..255]: byte table; T[256k + i]: slice-by-4 extension tables.
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ kCrcPoly : (c >> 1);
    T[i] = c;
  }
  __syncthreads();
  for (int t = 1; t < 4; t++) {
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
      const uint32_t prev = T[256 * (t - 1) + i];
      T[256 * t + i] = (prev >> 8) ^ T[prev & 0xffu];
    }
    __syncthreads();
  }
}

// One stream: `len` data bytes followed by `extra` virtual zero bytes (the
// filter block's type byte).
struct CrcStream {
  const uint8_t* data;
  const uint64_t* len_dev;  // device length (filter builds), or nullptr
  uint64_t len_host;        // used when len_dev == nullptr
  uint32_t extra;           // virtual trailing zero bytes
  uint32_t pad;
};

__device__ __forceinline__ uint64_t stream_len(const CrcStream& S) {
  return S.len_dev ? *S.len_dev : S.len_host;
}

struct XPowArg {
  uint32_t p[40];  // x^(2^k) mod P, k < 40
};

// Pass 1: raw CRC of each 64 KiB part (front-padded stream) -> partial[j][p].
__global__ __launch_bounds__(kCrcBlock) void crc_parts_kernel(const CrcStream* __restrict__ streams,
                                                              int max_parts, XPowArg xp,
                                                              uint32_t* __restrict__ partial) {
  __shared__ uint32_t T[1024];
  __shared__ uint32_t wv[kCrcBlock / 64];
  const int j = blockIdx.y;
  const uint32_t p = blockIdx.x;
  const CrcStream S = streams[j];
  const uint64_t len = stream_len(S);
  if (len == 0 && S.len_dev) {  // failed build (capacity): nothing to seal
    if (threadIdx.x == 0) partial[static_cast<uint64_t>(j) * max_parts + p] = 0;
    return;
  }
  const uint64_t total = len + S.extra;
  const uint64_t parts = (total + kCrcPart - 1) / kCrcPart;
  if (p >= parts) return;
  const uint64_t padded = parts * kCrcPart;
  const int64_t lead = static_cast<int64_t>(padded - total);  // zero bytes in front
  build_tables(T);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t acc = 0;
  for (uint32_t sub = 0; sub < kCrcSubs; sub++) {
    // this thread's 16 bytes: stream positions q .. q+15
    const int64_t q = static_cast<int64_t>(p * kCrcPart + sub * kCrcSub + threadIdx.x * 16u) - lead;
    uint32_t wd[4];
    if (q >= 0 && q + 16 <= static_cast<int64_t>(len) &&
        (reinterpret_cast<uintptr_t>(S.data + q) & 15u) == 0) {
      const uint4 v = *reinterpret_cast<const uint4*>(S.data + q);
      wd[0] = v.x; wd[1] = v.y; wd[2] = v.z; wd[3] = v.w;
    } else {
#pragma unroll
      for (int b4 = 0; b4 < 4; b4++) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int64_t d = q + 4 * b4 + b;
          const uint32_t byte = (d >= 0 && d < static_cast<int64_t>(len)) ? S.data[d] : 0u;
          x |= byte << (8 * b);
        }
        wd[b4] = x;
      }
    }
    uint32_t r = 0;
#pragma unroll
    for (int b4 = 0; b4 < 4; b4++) r = raw_word(r, wd[b4], T);
    // wave fold: level k joins 16*2^k-byte neighbours
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const uint32_t other = __shfl_xor(r, 1 << k, 64);
      if ((lane & (1 << k)) == 0) r = multmodp(r, xp.p[k + 7]) ^ other;  // x^(8*16*2^k)
    }
    if (lane == 0) wv[w] = r;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t s = 0;
      for (int q2 = 0; q2 < kCrcBlock / 64; q2++) s = multmodp(s, xp.p[3 + 10]) ^ wv[q2];  // 1 KiB steps
      acc = multmodp(acc, xp.p[3 + 14]) ^ s;  // 16 KiB steps
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[static_cast<uint64_t>(j) * max_parts + p] = acc;
}

// Pass 2: fold each stream's parts, finish the standard value, and either seal
// a filter block (type byte + masked crc, length += 5) or report the value.
__global__ void crc_finish_kernel(const CrcStream* __restrict__ streams, int n, int max_parts,
                                  XPowArg xp, const uint32_t* __restrict__ partial,
                                  uint8_t* const* __restrict__ seal_out,
                                  const uint64_t* __restrict__ seal_cap,
                                  uint64_t* __restrict__ seal_len, uint32_t* __restrict__ crc_out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const CrcStream S = streams[j];
  const uint64_t len = stream_len(S);
  if (seal_out && len == 0) return;  // failed build keeps out_len == 0
  const uint64_t total = len + S.extra;
  const uint64_t parts = (total + kCrcPart - 1) / kCrcPart;
  uint32_t raw = 0;
  for (uint64_t p = 0; p < parts; p++)
    raw = multmodp(raw, xp.p[3 + 16]) ^ partial[static_cast<uint64_t>(j) * max_parts + p];  // 64 KiB
  const uint32_t value = ~(multmodp(0xffffffffu, x8n(total, xp.p)) ^ raw);
  if (crc_out) crc_out[j] = value;
  if (seal_out) {
    if (len + 5 > seal_cap[j]) {
      seal_len[j] = 0;
      return;
    }
    const uint32_t m = ((value >> 15) | (value << 17)) + 0xa282ead8u;  // crc32c::Mask
    uint8_t* t = seal_out[j] + len;
    t[0] = 0;  // kNoCompression
    t[1] = static_cast<uint8_t>(m);
    t[2] = static_cast<uint8_t>(m >> 8);
    t[3] = static_cast<uint8_t>(m >> 16);
    t[4] = static_cast<uint8_t>(m >> 24);
    seal_len[j] = len + 5;
  }
}

XPowArg make_xpow() {
  XPowArg x;
  auto mul = [](uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int i = 0; i < 32; i++) {
      if (a & (0x80000000u >> i)) p ^= b;
      b = (b & 1u) ? (b >> 1) ^ kCrcPoly : (b >> 1);
    }
    return p;
  };
  x.p[0] = 0x40000000u;  // x^1
  for (int k = 1; k < 40; k++) x.p[k] = mul(x.p[k - 1], x.p[k - 1]);
  return x;
}

}  // namespace

uint64_t crc_max_parts(uint64_t max_len_plus_extra) {
  return (max_len_plus_extra + kCrcPart - 1) / kCrcPart;
}

hipError_t launch_crc_streams(const void* streams, int n, int max_parts, uint32_t* partial,
                              uint8_t* const* seal_out, const uint64_t* seal_cap, uint64_t* seal_len,
                              uint32_t* crc_out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  static const XPowArg xp = make_xpow();
  const CrcStream* st = static_cast<const CrcStream*>(streams);
  crc_parts_kernel<<<dim3(max_parts, n), kCrcBlock, 0, s>>>(st, max_parts, xp, partial);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  crc_finish_kernel<<<(n + 63) / 64, 64, 0, s>>>(st, n, max_parts, xp, partial, seal_out, seal_cap,
                                                 seal_len, crc_out);
  return hipGetLastError();
}

size_t crc_stream_size() { return sizeof(CrcStream); }

// Host tables of the fused seal (bloom_internal.h kCrcTabWords): slice-by-4
// tables, then powers x^(8n) mod P for the build slice's thread segments,
// whole slices and whole lines.
void full_block_crc_tables(int lgR, uint32_t* out) {
  auto mul = [](uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int i = 0; i < 32; i++) {
      if (a & (0x80000000u >> i)) p ^= b;
      b = (b & 1u) ? (b >> 1) ^ kCrcPoly : (b >> 1);
    }
    return p;
  };
  auto x8n = [&](uint64_t n) {  // x^(8n) by square-and-multiply
    uint32_t r = 0x80000000u, sq = 0x00800000u;  // x^0, x^8
    for (; n; n >>= 1, sq = mul(sq, sq))
      if (n & 1u) r = mul(r, sq);
    return r;
  };
  uint32_t* T = out;
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ kCrcPoly : (c >> 1);
    T[i] = c;
  }
  for (int t = 1; t < 4; t++)
    for (uint32_t i = 0; i < 256; i++) T[256 * t + i] = (T[256 * (t - 1) + i] >> 8) ^ T[T[256 * (t - 1) + i] & 0xffu];
  const uint64_t R = 1ull << lgR;
  const uint64_t seg = R * 64u / 512u;  // bytes per build-slice thread
  uint32_t* PS = out + 1024;
  const uint32_t step_s = x8n(seg);
  PS[0] = 0x80000000u;
  for (int m = 1; m < 512; m++) PS[m] = mul(PS[m - 1], step_s);
  uint32_t* P1 = PS + 512;
  const uint32_t step_1 = x8n(R * 64u);
  P1[0] = 0x80000000u;
  for (int m = 1; m < 256; m++) P1[m] = mul(P1[m - 1], step_1);
  uint32_t* P64 = P1 + 256;
  const uint32_t step_64 = x8n(64);
  P64[0] = 0x80000000u;
  for (int m = 1; m <= 2048; m++) P64[m] = mul(P64[m - 1], step_64);
}

void crc_stream_fill(void* dst, const uint8_t* data, const uint64_t* len_dev, uint64_t len_host,
                     uint32_t extra) {
  CrcStream* c = static_cast<CrcStream*>(dst);
  c->data = data;
  c->len_dev = len_dev;
  c->len_host = len_host;
  c->extra = extra;
  c->pad = 0;
}

}  // namespace dlsm
