// dlsm_amd/csrc/bloom_kernels.hip -- gfx950 (CDNA4) kernels for dLSM's Bloom
// filter hot path.  Integer/bit work only; no MFMA.  Wave64 throughout.
//
// Two kernel families produce byte-identical filters and masks:
//
//  * direct:  hash every key and set / test bits in the filter in global
//             memory (device-scope atomics for the build).  General: any key
//             shape, any filter set, any table size.
//  * sliced:  the LDS-tiled path.  A partition pass hashes each key once,
//             reads the 20-byte keys coalesced and buckets the 4-byte hashes
//             by filter slice (a run of R cache lines) inside its chunk; a
//             slice pass then gives every workgroup one slice in LDS, applies
//             (build: ds_or) or tests (probe: one ds_read_b64 per probe covers
//             8 stacked filters) all hashes of that slice, and streams the slice
//             out with 16-byte stores.  No global atomics, no random HBM
//             traffic: every HBM access is a coalesced stream.
//
// Semantics restated from (file:line in ruihong123/dLSM):
//   BloomHash                util/hash.cc:22-62, filter_policy.h:26-28
//   AddKey dedup             table/full_filter_block.cc:39-49
//   CalculateSpace / Finish  table/full_filter_block.cc:61-141
//   AddHash / HashMayMatch   util/bloom_impl.h:398-482 (LegacyLocality<false>)
//   legacy CreateFilter      util/bloom.cc:25-55, KeyMayMatch :57-81
#include <hip/hip_runtime.h>

#include "bloom_internal.h"

namespace dlsm {
namespace {

// ---------------------------------------------------------------------------
// Key hashing
// ---------------------------------------------------------------------------

// 20-byte key at a 4-byte-aligned address: 5 little-endian words, no tail.
__device__ __forceinline__ uint32_t hash_k20(const uint8_t* p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
  uint32_t h = hash_init(20, kBloomSeed);
  h = hash_word(h, __builtin_nontemporal_load(w + 0));
  h = hash_word(h, __builtin_nontemporal_load(w + 1));
  h = hash_word(h, __builtin_nontemporal_load(w + 2));
  h = hash_word(h, __builtin_nontemporal_load(w + 3));
  h = hash_word(h, __builtin_nontemporal_load(w + 4));
  return h;
}

// Any length, any alignment: aligned dword loads + v_alignbyte.  Never reads a
// dword that holds no byte of the key.
__device__ uint32_t hash_bytes(const uint8_t* p, uint64_t len) {
  uint32_t h = hash_init(len, kBloomSeed);
  const uint64_t nw = len >> 2;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t sh = static_cast<uint32_t>(a & 3u);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a - sh);
  if (nw) {
    if (sh == 0) {
      for (uint64_t i = 0; i < nw; i++) h = hash_word(h, w[i]);
    } else {
      uint32_t lo = w[0];
      for (uint64_t i = 0; i < nw; i++) {
        const uint32_t hi = w[i + 1];
        h = hash_word(h, __builtin_amdgcn_alignbyte(hi, lo, sh));
        lo = hi;
      }
    }
  }
  const uint32_t rem = static_cast<uint32_t>(len & 3u);
  uint32_t t = 0;
  for (uint32_t j = 0; j < rem; j++) t |= uint32_t(p[4 * nw + j]) << (8 * j);
  return hash_tail(h, t, rem);
}

template <int MODE>
__device__ __forceinline__ uint32_t key_hash(const KeyDesc& kd, uint64_t i) {
  if constexpr (MODE == KM_K20) {
    return hash_k20(kd.bytes + i * 20u);
  } else {
    uint64_t s, l;
    if (kd.offsets) {
      s = kd.offsets[i];
      l = kd.offsets[i + 1] - s;
    } else {
      s = i * kd.key_len;
      l = kd.key_len;
    }
    return hash_bytes(kd.bytes + s, l);
  }
}

// ---------------------------------------------------------------------------
// Block helpers (256 threads = 4 waves of 64)
// ---------------------------------------------------------------------------

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// In-place exclusive scan of a[0, n) (n <= 4*kBlock) held in LDS.  Callers
// synchronise before (a written by other threads); returns the total and ends
// with a barrier.
__device__ uint32_t block_excl_scan_lds(uint32_t* a, int n, uint32_t* wsum) {
  const int t = threadIdx.x;
  uint32_t v[4];
  uint32_t local = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int idx = 4 * t + q;
    v[q] = idx < n ? a[idx] : 0u;
    local += v[q];
  }
  const uint32_t incl = wave_incl_scan(local);
  const int lane = t & 63, w = t >> 6;
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint32_t base = 0, total = 0;
#pragma unroll
  for (int ww = 0; ww < kBlock / 64; ww++) {
    const uint32_t x = wsum[ww];
    if (ww < w) base += x;
    total += x;
  }
  uint32_t run = base + incl - local;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int idx = 4 * t + q;
    if (idx < n) a[idx] = run;
    run += v[q];
  }
  __syncthreads();
  return total;
}

__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* wsum) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int w = 0; w < kBlock / 64; w++) t += wsum[w];
  __syncthreads();
  return t;
}

// Largest j with starts[j] <= b (starts non-decreasing, starts[0] == 0).
template <typename T>
__device__ __forceinline__ int find_job(const T* starts, int n_jobs, T b) {
  int lo = 0, hi = n_jobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (starts[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Largest c in [0, n) with pre[c] <= e (pre[0] == 0 <= e).
__device__ __forceinline__ int seg_search(const uint32_t* pre, int n, uint32_t e) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pre[mid] <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// LegacyLocalityBloomImpl<false>::AddHash into one 64-byte line held as 16
// LDS words (bloom_impl.h:427-443).
__device__ __forceinline__ void lds_add_hash(uint32_t* line, uint32_t h, int k) {
  const uint32_t delta = bloom_delta(h);
  for (int i = 0; i < k; i++) {
    const uint32_t bp = h & 511u;
    atomicOr(&line[bp >> 5], 1u << (bp & 31u));
    h += delta;
  }
}

// Filter trailer (full_filter_block.cc:133-135): k byte + Fixed32 num_lines.
__device__ __forceinline__ void write_trailer(uint8_t* out, uint32_t L, int k) {
  uint8_t* t = out + static_cast<uint64_t>(L) * 64u;
  t[0] = static_cast<uint8_t>(static_cast<int8_t>(k));
  t[1] = static_cast<uint8_t>(L);
  t[2] = static_cast<uint8_t>(L >> 8);
  t[3] = static_cast<uint8_t>(L >> 16);
  t[4] = static_cast<uint8_t>(L >> 24);
}

// ---------------------------------------------------------------------------
// Full filter build: hash + consecutive-dedup count (+ slice partition)
// One workgroup per chunk of kBuildChunk keys of one job.
// ---------------------------------------------------------------------------
template <int MODE, bool PART>
__global__ __launch_bounds__(kBlock) void full_partition_kernel(
    const FullJobDev* __restrict__ jobs, const uint32_t* __restrict__ chunk0s, int n_jobs,
    JobState* __restrict__ st, uint32_t* __restrict__ entries, uint32_t* __restrict__ tab,
    int lgR) {
  constexpr int C = kBuildChunk;
  constexpr int PER = C / kBlock;
  __shared__ uint32_t hs[C + 1];
  __shared__ uint32_t hist[kMaxSlices + 1];
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ int sj;
  const int tid = threadIdx.x;
  if (tid == 0) sj = find_job(chunk0s, n_jobs, static_cast<uint32_t>(blockIdx.x));
  __syncthreads();
  const int j = sj;
  const FullJobDev J = jobs[j];
  const uint32_t c = blockIdx.x - J.chunk0;
  const uint64_t first = static_cast<uint64_t>(c) * C;
  const uint64_t left = J.keys.n - first;
  const uint32_t nk = left < static_cast<uint64_t>(C) ? static_cast<uint32_t>(left) : C;

  uint32_t h[PER];
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const uint32_t i = r * kBlock + tid;
    h[r] = 0;
    if (i < nk) {
      h[r] = key_hash<MODE>(J.keys, first + i);
      hs[i + 1] = h[r];
    }
  }
  if (tid == 0) hs[0] = first > 0 ? key_hash<MODE>(J.keys, first - 1) : ~h[0];
  __syncthreads();
  // AddKey (full_filter_block.cc:45-48): a hash counts unless it equals the
  // immediately preceding one; the job's key 0 always counts (hs[0] = ~h).
  uint32_t cnt = 0;
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const uint32_t i = r * kBlock + tid;
    if (i < nk) cnt += (hs[i + 1] != hs[i]) ? 1u : 0u;
  }
  cnt = block_sum(cnt, wsum);
  if (tid == 0) atomicAdd(&st[j].distinct, static_cast<unsigned long long>(cnt));
  if constexpr (!PART) return;

  const uint32_t S = J.n_slices;
  for (uint32_t b = tid; b <= S; b += kBlock) hist[b] = 0;
  __syncthreads();
  uint32_t code[PER];
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const uint32_t i = r * kBlock + tid;
    if (i < nk) {
      const uint32_t s = fastmod(h[r], J.L_spec, J.magic_spec) >> lgR;
      const uint32_t rank = atomicAdd(&hist[s], 1u);
      code[r] = (rank << 9) | s;
    }
  }
  __syncthreads();
  block_excl_scan_lds(hist, static_cast<int>(S + 1), wsum);
  for (uint32_t b = tid; b <= S; b += kBlock)
    tab[J.tab0 + static_cast<uint64_t>(b) * J.n_chunks + c] = hist[b];
  uint32_t* ent = entries + J.entry0 + first;
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const uint32_t i = r * kBlock + tid;
    if (i < nk) ent[hist[code[r] & 511u] + (code[r] >> 9)] = h[r];
  }
}

// ---------------------------------------------------------------------------
// Full filter build, sliced: one workgroup per (job, slice of 2^LGR lines).
// ---------------------------------------------------------------------------
template <int LGR>
__global__ __launch_bounds__(kBlock) void full_slice_kernel(
    const FullJobDev* __restrict__ jobs, const uint32_t* __restrict__ slice0s, int n_jobs,
    JobState* __restrict__ st, const uint32_t* __restrict__ entries,
    const uint32_t* __restrict__ tab) {
  constexpr uint32_t R = 1u << LGR;
  __shared__ __attribute__((aligned(16))) uint32_t sl[R * 16];
  __shared__ uint32_t g_off[kBlock];
  __shared__ uint32_t g_pre[kBlock + 1];
  __shared__ uint32_t wsum[kBlock / 64];
  __shared__ int sj;
  const int tid = threadIdx.x;
  if (tid == 0) sj = find_job(slice0s, n_jobs, static_cast<uint32_t>(blockIdx.x));
  __syncthreads();
  const int j = sj;
  const FullJobDev J = jobs[j];
  const uint32_t s = blockIdx.x - J.slice0;
  uint32_t total_bits;
  const uint32_t L = full_num_lines(st[j].distinct, J.bpk, &total_bits);
  const uint64_t len = static_cast<uint64_t>(total_bits / 8u) + 5u;
  if (len > J.out_cap) {
    if (s == 0 && tid == 0) {
      *J.out_len = 0;
      st[j].status = -2;
    }
    return;
  }
  const uint32_t lo_line = s << LGR;
  for (uint32_t w = tid; w < R * 16; w += kBlock) sl[w] = 0;
  __syncthreads();
  if (L != 0 && lo_line < L) {
    const uint32_t magic = fastmod_magic(L);
    if (L == J.L_spec) {
      const uint32_t nC = J.n_chunks;
      const uint32_t* row0 = tab + J.tab0 + static_cast<uint64_t>(s) * nC;
      const uint32_t* row1 = row0 + nC;
      for (uint32_t g0 = 0; g0 < nC; g0 += kBlock) {
        const uint32_t gc = min(static_cast<uint32_t>(kBlock), nC - g0);
        if (tid < gc) {
          const uint32_t o0 = row0[g0 + tid];
          g_off[tid] = o0;
          g_pre[tid] = row1[g0 + tid] - o0;
        } else {
          g_pre[tid] = 0;
        }
        __syncthreads();
        const uint32_t T = block_excl_scan_lds(g_pre, kBlock, wsum);
        const uint32_t* ent = entries + J.entry0 + static_cast<uint64_t>(g0) * kBuildChunk;
        for (uint32_t e = tid; e < T; e += kBlock) {
          const int cc = seg_search(g_pre, static_cast<int>(gc), e);
          const uint32_t hv =
              ent[static_cast<uint64_t>(cc) * kBuildChunk + g_off[cc] + (e - g_pre[cc])];
          const uint32_t li = fastmod(hv, L, magic) - lo_line;
          lds_add_hash(sl + li * 16u, hv, J.k);
        }
        __syncthreads();
      }
    } else {
      // Duplicates lowered the line count below the speculative one: the
      // partition used the wrong modulus, so scan every hash of the job.
      const uint32_t* ent = entries + J.entry0;
      for (uint64_t e = tid; e < J.keys.n; e += kBlock) {
        const uint32_t hv = ent[e];
        const uint32_t line = fastmod(hv, L, magic);
        if ((line >> LGR) == s) lds_add_hash(sl + (line - lo_line) * 16u, hv, J.k);
      }
    }
    __syncthreads();
    const uint32_t nl = min(R, L - lo_line);
    uint4* dst = reinterpret_cast<uint4*>(J.out + static_cast<uint64_t>(lo_line) * 64u);
    const uint4* src = reinterpret_cast<const uint4*>(sl);
    for (uint32_t w = tid; w < nl * 4u; w += kBlock) dst[w] = src[w];
  }
  if (s == 0 && tid == 0) {
    write_trailer(J.out, L, J.k);
    *J.out_len = len;
  }
}

// ---------------------------------------------------------------------------
// Full filter build, direct path: zero + trailer, then global-atomic scatter.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void full_zero_kernel(const FullJobDev* __restrict__ jobs,
                                                           JobState* __restrict__ st) {
  const FullJobDev J = jobs[blockIdx.y];
  uint32_t total_bits;
  const uint32_t L = full_num_lines(st[blockIdx.y].distinct, J.bpk, &total_bits);
  const uint64_t len = static_cast<uint64_t>(total_bits / 8u) + 5u;
  if (len > J.out_cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      *J.out_len = 0;
      st[blockIdx.y].status = -2;
    }
    return;
  }
  uint32_t* o = reinterpret_cast<uint32_t*>(J.out);
  const uint64_t words = static_cast<uint64_t>(L) * 16u;
  for (uint64_t w = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x; w < words;
       w += static_cast<uint64_t>(gridDim.x) * kBlock)
    o[w] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    write_trailer(J.out, L, J.k);
    *J.out_len = len;
  }
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void full_scatter_kernel(
    const FullJobDev* __restrict__ jobs, const uint32_t* __restrict__ chunk0s, int n_jobs,
    const JobState* __restrict__ st) {
  __shared__ int sj;
  if (threadIdx.x == 0) sj = find_job(chunk0s, n_jobs, static_cast<uint32_t>(blockIdx.x));
  __syncthreads();
  const int j = sj;
  if (st[j].status != 0) return;
  const FullJobDev J = jobs[j];
  const uint32_t L = full_num_lines(st[j].distinct, J.bpk, nullptr);
  if (L == 0) return;
  const uint32_t magic = fastmod_magic(L);
  const uint64_t first = static_cast<uint64_t>(blockIdx.x - J.chunk0) * kBuildChunk;
  const uint64_t end = min(J.keys.n, first + kBuildChunk);
  uint32_t* o = reinterpret_cast<uint32_t*>(J.out);
  for (uint64_t i = first + threadIdx.x; i < end; i += kBlock) {
    uint32_t h = key_hash<MODE>(J.keys, i);
    uint32_t* line = o + static_cast<uint64_t>(fastmod(h, L, magic)) * 16u;
    const uint32_t delta = bloom_delta(h);
    for (int q = 0; q < J.k; q++) {
      const uint32_t bp = h & 511u;
      atomicOr(&line[bp >> 5], 1u << (bp & 31u));
      h += delta;
    }
  }
}

// ---------------------------------------------------------------------------
// Full filter probe, direct: one thread per key, global reads of the filters.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t full_may_match(uint32_t h, const FilterDev& f) {
  // FullFilterBlockReader::KeyMayMatch (full_filter_block.cc:269-284).
  const uint32_t off = fastmod(h, f.L, f.magic) << f.lg;  // u32 like GetLine << lg
  const uint32_t delta = bloom_delta(h);
  if (f.lg == 6) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(f.data + off);
    for (int i = 0; i < f.k; i++) {
      const uint32_t bp = h & 511u;
      if (((w[bp >> 5] >> (bp & 31u)) & 1u) == 0) return 0;
      h += delta;
    }
  } else {  // log2_cache_line_size_ == 0: one-byte "lines" (full_filter_block.h:85)
    const uint32_t b = f.data[off];
    for (int i = 0; i < f.k; i++) {
      if (((b >> (h & 7u)) & 1u) == 0) return 0;
      h += delta;
    }
  }
  return 1;
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void probe_direct_kernel(const FilterDev* __restrict__ fs,
                                                              int F, KeyDesc kd,
                                                              uint8_t* __restrict__ mask) {
  __shared__ FilterDev sf[64];
  for (int f = threadIdx.x; f < F; f += kBlock) sf[f] = fs[f];
  __syncthreads();
  const int mb = (F + 7) >> 3;
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x; i < kd.n;
       i += static_cast<uint64_t>(gridDim.x) * kBlock) {
    const uint32_t h = key_hash<MODE>(kd, i);
    for (int g = 0; g < mb; g++) {
      uint32_t m = 0;
      const int fe = min(F, 8 * g + 8);
      for (int f = 8 * g; f < fe; f++) m |= full_may_match(h, sf[f]) << (f - 8 * g);
      mask[i * mb + g] = static_cast<uint8_t>(m);
    }
  }
}

// ---------------------------------------------------------------------------
// Full filter probe, sliced (F <= 8 filters with a common line count / k).
// Stacked image: u64 word (line*64 + byte) holds byte `byte` of filter f in
// its byte f, so one 8-byte LDS read answers a probe for all 8 filters.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void stack_filters_kernel(const FilterDev* __restrict__ fs,
                                                               int F, uint64_t words,
                                                               uint64_t* __restrict__ stacked) {
  for (uint64_t w = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x; w < words;
       w += static_cast<uint64_t>(gridDim.x) * kBlock) {
    uint64_t v = 0;
    for (int f = 0; f < F; f++) v |= static_cast<uint64_t>(fs[f].data[w]) << (8 * f);
    stacked[w] = v;
  }
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void probe_partition_kernel(
    KeyDesc kd, uint32_t L, uint32_t magic, int lgR, uint32_t S, uint32_t nC,
    uint32_t* __restrict__ entries, uint16_t* __restrict__ pos, uint32_t* __restrict__ tab) {
  constexpr int C = kProbeChunk;
  constexpr int PER = C / kBlock;
  __shared__ uint32_t hist[kMaxSlices + 1];
  __shared__ uint32_t wsum[kBlock / 64];
  const int tid = threadIdx.x;
  const uint32_t c = blockIdx.x;
  const uint64_t first = static_cast<uint64_t>(c) * C;
  const uint64_t left = kd.n - first;
  const uint32_t nk = left < static_cast<uint64_t>(C) ? static_cast<uint32_t>(left) : C;
  for (uint32_t b = tid; b <= S; b += kBlock) hist[b] = 0;
  __syncthreads();
  uint32_t h[PER], code[PER];
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const uint32_t i = r * kBlock + tid;
    if (i < nk) {
      h[r] = key_hash<MODE>(kd, first + i);
      const uint32_t s = fastmod(h[r], L, magic) >> lgR;
      const uint32_t rank = atomicAdd(&hist[s], 1u);
      code[r] = (rank << 9) | s;
    }
  }
  __syncthreads();
  block_excl_scan_lds(hist, static_cast<int>(S + 1), wsum);
  for (uint32_t b = tid; b <= S; b += kBlock) tab[static_cast<uint64_t>(b) * nC + c] = hist[b];
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const uint32_t i = r * kBlock + tid;
    if (i < nk) {
      const uint32_t p = hist[code[r] & 511u] + (code[r] >> 9);
      entries[first + p] = h[r];
      pos[first + i] = static_cast<uint16_t>(p);
    }
  }
}

template <int LGR>
__global__ __launch_bounds__(kBlock) void probe_slice_kernel(
    const uint64_t* __restrict__ stacked, uint32_t L, uint32_t magic, int k, uint32_t S,
    uint32_t nC, const uint32_t* __restrict__ entries, const uint32_t* __restrict__ tab,
    uint8_t* __restrict__ smask, int parts) {
  constexpr uint32_t R = 1u << LGR;
  __shared__ uint64_t sl[R * 64];
  __shared__ uint32_t g_off[kBlock];
  __shared__ uint32_t g_pre[kBlock + 1];
  __shared__ uint32_t wsum[kBlock / 64];
  const int tid = threadIdx.x;
  const uint32_t s = blockIdx.x % S;
  const uint32_t p = blockIdx.x / S;
  const uint32_t lo_line = s << LGR;
  const uint32_t nl = min(R, L - lo_line);
  const uint64_t* src = stacked + static_cast<uint64_t>(lo_line) * 64u;
  for (uint32_t w = tid; w < nl * 64u; w += kBlock) sl[w] = src[w];
  const uint32_t c_lo = static_cast<uint32_t>(static_cast<uint64_t>(p) * nC / parts);
  const uint32_t c_hi = static_cast<uint32_t>(static_cast<uint64_t>(p + 1) * nC / parts);
  const uint32_t* row0 = tab + static_cast<uint64_t>(s) * nC;
  const uint32_t* row1 = row0 + nC;
  __syncthreads();
  for (uint32_t g0 = c_lo; g0 < c_hi; g0 += kBlock) {
    const uint32_t gc = min(static_cast<uint32_t>(kBlock), c_hi - g0);
    if (tid < gc) {
      const uint32_t o0 = row0[g0 + tid];
      g_off[tid] = o0;
      g_pre[tid] = row1[g0 + tid] - o0;
    } else {
      g_pre[tid] = 0;
    }
    __syncthreads();
    const uint32_t T = block_excl_scan_lds(g_pre, kBlock, wsum);
    const uint64_t base = static_cast<uint64_t>(g0) * kProbeChunk;
    for (uint32_t e = tid; e < T; e += kBlock) {
      const int cc = seg_search(g_pre, static_cast<int>(gc), e);
      const uint64_t idx = base + static_cast<uint64_t>(cc) * kProbeChunk + g_off[cc] + (e - g_pre[cc]);
      uint32_t hv = entries[idx];
      const uint32_t li = fastmod(hv, L, magic) - lo_line;
      const uint64_t* line = sl + li * 64u;
      const uint32_t delta = bloom_delta(hv);
      uint64_t acc = 0x0101010101010101ull;
      for (int q = 0; q < k; q++) {
        const uint32_t bp = hv & 511u;
        acc &= line[bp >> 3] >> (bp & 7u);
        hv += delta;
      }
      acc &= 0x0101010101010101ull;
      smask[idx] = static_cast<uint8_t>((acc * 0x0102040810204080ull) >> 56);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void probe_unpermute_kernel(uint64_t n,
                                                                 const uint16_t* __restrict__ pos,
                                                                 const uint8_t* __restrict__ smask,
                                                                 uint8_t* __restrict__ mask) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * kBlock) {
    const uint64_t base = i & ~static_cast<uint64_t>(kProbeChunk - 1);
    mask[i] = smask[base + pos[i]];
  }
}

// ---------------------------------------------------------------------------
// Legacy FilterPolicy format (util/bloom.cc): global double hashing.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t legacy_bitpos(uint32_t h, uint64_t bits, uint32_t magic) {
  // bitpos = h % bits (size_t); for bits >= 2^32 that is h itself.
  return bits > 0xffffffffull ? h : fastmod(h, static_cast<uint32_t>(bits), magic);
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void legacy_scatter_kernel(
    const LegacyJobDev* __restrict__ jobs, const uint64_t* __restrict__ key0s, int n_jobs,
    uint64_t total) {
  __shared__ uint64_t sk[256];
  for (int t = threadIdx.x; t < n_jobs; t += kBlock) sk[t] = key0s[t];
  __syncthreads();
  for (uint64_t g = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x; g < total;
       g += static_cast<uint64_t>(gridDim.x) * kBlock) {
    const int j = find_job(sk, n_jobs, g);
    const LegacyJobDev& J = jobs[j];
    uint32_t h = key_hash<MODE>(J.keys, g - J.key0);
    const uint32_t delta = bloom_delta(h);
    uint32_t* o = reinterpret_cast<uint32_t*>(J.out);
    for (int q = 0; q < J.k; q++) {
      const uint32_t bp = legacy_bitpos(h, J.bits, J.magic);
      atomicOr(&o[bp >> 5], 1u << (bp & 31u));
      h += delta;
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void legacy_probe_kernel(const uint8_t* __restrict__ filter,
                                                              uint64_t bits, uint32_t magic, int k,
                                                              int trivial, KeyDesc kd,
                                                              uint8_t* __restrict__ out) {
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x; i < kd.n;
       i += static_cast<uint64_t>(gridDim.x) * kBlock) {
    uint8_t r;
    if (trivial) {
      r = trivial == 2 ? 1 : 0;
    } else {
      uint32_t h = key_hash<MODE>(kd, i);
      const uint32_t delta = bloom_delta(h);
      r = 1;
      for (int q = 0; q < k; q++) {
        const uint32_t bp = legacy_bitpos(h, bits, magic);
        if (((filter[bp >> 3] >> (bp & 7u)) & 1u) == 0) {
          r = 0;
          break;
        }
        h += delta;
      }
    }
    out[i] = r;
  }
}

inline unsigned grid_for(uint64_t n, unsigned cap = 256u * 16u) {
  const uint64_t g = (n + kBlock - 1) / kBlock;
  return static_cast<unsigned>(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
hipError_t launch_full_count(const FullJobDev* jobs, const uint32_t* chunk0s, int n_jobs,
                             uint32_t total_chunks, JobState* st, int mode, hipStream_t s) {
  if (total_chunks == 0) return hipSuccess;
  if (mode == KM_K20)
    full_partition_kernel<KM_K20, false><<<total_chunks, kBlock, 0, s>>>(jobs, chunk0s, n_jobs, st,
                                                                          nullptr, nullptr, 0);
  else
    full_partition_kernel<KM_GENERIC, false><<<total_chunks, kBlock, 0, s>>>(
        jobs, chunk0s, n_jobs, st, nullptr, nullptr, 0);
  return hipGetLastError();
}

hipError_t launch_full_zero(const FullJobDev* jobs, const uint32_t*, int n_jobs, uint32_t,
                            JobState* st, hipStream_t s) {
  if (n_jobs == 0) return hipSuccess;
  full_zero_kernel<<<dim3(64, n_jobs), kBlock, 0, s>>>(jobs, st);
  return hipGetLastError();
}

hipError_t launch_full_scatter(const FullJobDev* jobs, const uint32_t* chunk0s, int n_jobs,
                               uint32_t total_chunks, JobState* st, int mode, hipStream_t s) {
  if (total_chunks == 0) return hipSuccess;
  if (mode == KM_K20)
    full_scatter_kernel<KM_K20><<<total_chunks, kBlock, 0, s>>>(jobs, chunk0s, n_jobs, st);
  else
    full_scatter_kernel<KM_GENERIC><<<total_chunks, kBlock, 0, s>>>(jobs, chunk0s, n_jobs, st);
  return hipGetLastError();
}

hipError_t launch_full_finalize(const FullJobDev*, int, JobState*, hipStream_t) {
  return hipSuccess;
}

hipError_t launch_full_partition(const FullJobDev* jobs, const uint32_t* chunk0s, int n_jobs,
                                 uint32_t total_chunks, JobState* st, uint32_t* entries,
                                 uint32_t* tab, int lgR, int mode, hipStream_t s) {
  if (total_chunks == 0) return hipSuccess;
  if (mode == KM_K20)
    full_partition_kernel<KM_K20, true><<<total_chunks, kBlock, 0, s>>>(jobs, chunk0s, n_jobs, st,
                                                                         entries, tab, lgR);
  else
    full_partition_kernel<KM_GENERIC, true><<<total_chunks, kBlock, 0, s>>>(
        jobs, chunk0s, n_jobs, st, entries, tab, lgR);
  return hipGetLastError();
}

hipError_t launch_full_slices(const FullJobDev* jobs, const uint32_t* slice0s, int n_jobs,
                              uint32_t total_slices, JobState* st, const uint32_t* entries,
                              const uint32_t* tab, int lgR, hipStream_t s) {
  if (total_slices == 0) return hipSuccess;
  switch (lgR) {
    case 8:
      full_slice_kernel<8><<<total_slices, kBlock, 0, s>>>(jobs, slice0s, n_jobs, st, entries, tab);
      break;
    case 9:
      full_slice_kernel<9><<<total_slices, kBlock, 0, s>>>(jobs, slice0s, n_jobs, st, entries, tab);
      break;
    case 10:
      full_slice_kernel<10><<<total_slices, kBlock, 0, s>>>(jobs, slice0s, n_jobs, st, entries, tab);
      break;
    case 11:
      full_slice_kernel<11><<<total_slices, kBlock, 0, s>>>(jobs, slice0s, n_jobs, st, entries, tab);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_probe_direct(const FilterDev* fs, int n_filters, KeyDesc keys, uint8_t* mask,
                               int mode, hipStream_t s) {
  if (keys.n == 0) return hipSuccess;
  const unsigned g = grid_for(keys.n, 256u * 64u);
  if (mode == KM_K20)
    probe_direct_kernel<KM_K20><<<g, kBlock, 0, s>>>(fs, n_filters, keys, mask);
  else
    probe_direct_kernel<KM_GENERIC><<<g, kBlock, 0, s>>>(fs, n_filters, keys, mask);
  return hipGetLastError();
}

hipError_t launch_stack_filters(const FilterDev* fs, int n_filters, uint32_t L, uint64_t* stacked,
                                hipStream_t s) {
  const uint64_t words = static_cast<uint64_t>(L) * 64u;
  stack_filters_kernel<<<grid_for(words), kBlock, 0, s>>>(fs, n_filters, words, stacked);
  return hipGetLastError();
}

hipError_t launch_probe_partition(KeyDesc keys, uint32_t L, uint32_t magic, int lgR,
                                  uint32_t n_slices, uint32_t* entries, uint16_t* pos,
                                  uint32_t* tab, int mode, hipStream_t s) {
  const uint32_t nC = static_cast<uint32_t>((keys.n + kProbeChunk - 1) / kProbeChunk);
  if (nC == 0) return hipSuccess;
  if (mode == KM_K20)
    probe_partition_kernel<KM_K20><<<nC, kBlock, 0, s>>>(keys, L, magic, lgR, n_slices, nC,
                                                         entries, pos, tab);
  else
    probe_partition_kernel<KM_GENERIC><<<nC, kBlock, 0, s>>>(keys, L, magic, lgR, n_slices, nC,
                                                             entries, pos, tab);
  return hipGetLastError();
}

hipError_t launch_probe_slices(const uint64_t* stacked, uint32_t L, uint32_t magic, int k, int lgR,
                               uint32_t n_slices, uint32_t n_chunks, uint64_t,
                               const uint32_t* entries, const uint32_t* tab, uint8_t* smask,
                               int parts, hipStream_t s) {
  if (n_chunks == 0) return hipSuccess;
  if (lgR != 7) return hipErrorInvalidValue;
  probe_slice_kernel<7><<<n_slices * parts, kBlock, 0, s>>>(stacked, L, magic, k, n_slices,
                                                            n_chunks, entries, tab, smask, parts);
  return hipGetLastError();
}

hipError_t launch_probe_unpermute(uint64_t n_keys, const uint16_t* pos, const uint8_t* smask,
                                  uint8_t* mask, hipStream_t s) {
  if (n_keys == 0) return hipSuccess;
  probe_unpermute_kernel<<<grid_for(n_keys, 256u * 64u), kBlock, 0, s>>>(n_keys, pos, smask, mask);
  return hipGetLastError();
}

hipError_t launch_legacy_scatter(const LegacyJobDev* jobs, const uint64_t* key0s, int n_jobs,
                                 uint64_t total_keys, int mode, hipStream_t s) {
  if (total_keys == 0) return hipSuccess;
  const unsigned g = grid_for(total_keys, 256u * 64u);
  if (mode == KM_K20)
    legacy_scatter_kernel<KM_K20><<<g, kBlock, 0, s>>>(jobs, key0s, n_jobs, total_keys);
  else
    legacy_scatter_kernel<KM_GENERIC><<<g, kBlock, 0, s>>>(jobs, key0s, n_jobs, total_keys);
  return hipGetLastError();
}

hipError_t launch_legacy_probe(const uint8_t* filter, uint64_t bits, uint32_t magic, int k,
                               int trivial, KeyDesc keys, uint8_t* out, int mode, hipStream_t s) {
  if (keys.n == 0) return hipSuccess;
  const unsigned g = grid_for(keys.n, 256u * 64u);
  if (mode == KM_K20)
    legacy_probe_kernel<KM_K20><<<g, kBlock, 0, s>>>(filter, bits, magic, k, trivial, keys, out);
  else
    legacy_probe_kernel<KM_GENERIC><<<g, kBlock, 0, s>>>(filter, bits, magic, k, trivial, keys, out);
  return hipGetLastError();
}

}  // namespace dlsm
