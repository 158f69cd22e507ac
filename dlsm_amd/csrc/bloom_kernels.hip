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

#include <algorithm>
#include <atomic>
#include <cstdlib>

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
  } else if constexpr (MODE == KM_K28) {
    return hash_k20(kd.bytes + i * 28u);  // ExtractUserKey: the first 20 of 28 bytes
  } else if constexpr (MODE == KM_HASH) {
    return reinterpret_cast<const uint32_t*>(kd.bytes)[i];
  } else {
    uint64_t s, l;
    if (kd.offsets) {
      s = kd.offsets[i];
      l = kd.offsets[i + 1] - s;
    } else {
      s = i * kd.key_len;
      l = kd.key_len;
    }
    l = l > kd.suffix ? l - kd.suffix : 0;  // ExtractUserKey (db/dbformat.h:374-377)
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

// In-place exclusive scan of a[0, n) (n <= 4*NT) held in LDS by an NT-thread
// block.  Callers synchronise before (a written by other threads); returns the
// total and ends with a barrier.
template <int NT>
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
  for (int ww = 0; ww < NT / 64; ww++) {
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

// XCD-aware block order.  Workgroups are dispatched to the 8 XCDs
// round-robin (block b -> XCD b % 8; a speed assumption only, results never
// depend on it).  Renumber so each XCD gets one contiguous run of work items:
// adjacent slices read adjacent bucket segments of every chunk (and write
// adjacent answer bytes), so running them on one XCD turns the cache lines
// they share into L2 hits / whole-line writes instead of one fetch per XCD.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, j = b >> 3, q = n >> 3, r = n & 7u;
  return x * q + min(x, r) + j;
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

template <int K>
__device__ __forceinline__ void lds_add_hash_k(uint32_t* line, uint32_t h) {
  const uint32_t delta = bloom_delta(h);
#pragma unroll
  for (int i = 0; i < K; i++) {
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
// Chunk hashing.  Key i of a chunk (i = r*NT + t) is hashed by thread t into
// h[r].  K20: the chunk's bytes are staged through LDS in tiles of
// TILE = 4*NT keys with 16-byte, fully coalesced global loads (double-buffered
// in registers), then each thread reads its key's five dwords from LDS (stride
// 5 dwords: conflict-free).  GENERIC: each thread hashes its keys directly.
// ---------------------------------------------------------------------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// A 16-byte store through a global-address-space pointer.  Output pointers
// read from a job descriptor are generic, and generic (flat) stores count in
// lgkmcnt as well as vmcnt: the next LDS wait then waits for the stores to
// complete (the slice passes' LDS -> HBM loops serialised on store latency).
typedef __attribute__((address_space(1))) u32x4 g_u32x4_w;
__device__ __forceinline__ void st_global16(void* p, uint4 v) {
  *(g_u32x4_w*)(reinterpret_cast<uintptr_t>(p)) = u32x4{v.x, v.y, v.z, v.w};
}
typedef __attribute__((address_space(1))) uint8_t g_u8_w;
__device__ __forceinline__ void st_global1(void* p, uint8_t v) { *(g_u8_w*)(reinterpret_cast<uintptr_t>(p)) = v; }

template <int NT, int KPT, int KB = 20>
struct K20Tile {
  static constexpr int kKeys = KPT * NT;                 // keys per tile
  static constexpr int kVec = kKeys * KB / 16;           // uint4 per tile
  static constexpr int kPer = (kVec + NT - 1) / NT;      // uint4 per thread
};

template <int NT, int KPT, int KB = 20>
__device__ __forceinline__ void k20_tile_fetch(const uint8_t* base, uint32_t nbytes, int q,
                                               uint4 (&r)[K20Tile<NT, KPT, KB>::kPer]) {
  using TL = K20Tile<NT, KPT, KB>;
  const uint4* b4 = reinterpret_cast<const uint4*>(base) + q * TL::kVec;
  const uint32_t tile_off = q * TL::kVec * 16u;
#pragma unroll
  for (int v = 0; v < TL::kPer; v++) {
    const uint32_t u = v * NT + threadIdx.x;
    if (TL::kVec % NT != 0 && u >= static_cast<uint32_t>(TL::kVec)) break;
    const uint32_t off = tile_off + u * 16u;
    if (off + 16u <= nbytes) {
      const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b4 + u));
      r[v] = make_uint4(x.x, x.y, x.z, x.w);
    } else {
      // tail: dword-granular (nbytes is a multiple of 4), never past the keys
      const uint32_t* d = reinterpret_cast<const uint32_t*>(base + off);
      r[v].x = off + 4u <= nbytes ? d[0] : 0u;
      r[v].y = off + 8u <= nbytes ? d[1] : 0u;
      r[v].z = off + 12u <= nbytes ? d[2] : 0u;
      r[v].w = 0u;
    }
  }
}

template <int NT, int KPT, int KB = 20>
__device__ __forceinline__ void k20_tile_store(uint4* lds, const uint4 (&r)[K20Tile<NT, KPT, KB>::kPer]) {
  using TL = K20Tile<NT, KPT, KB>;
#pragma unroll
  for (int v = 0; v < TL::kPer; v++) {
    const uint32_t u = v * NT + threadIdx.x;
    if (TL::kVec % NT != 0 && u >= static_cast<uint32_t>(TL::kVec)) break;
    lds[u] = r[v];
  }
}

__device__ __forceinline__ uint32_t hash_k20_lds(const uint32_t* w) {
  uint32_t h = hash_init(20, kBloomSeed);
  h = hash_word(h, w[0]);
  h = hash_word(h, w[1]);
  h = hash_word(h, w[2]);
  h = hash_word(h, w[3]);
  h = hash_word(h, w[4]);
  return h;
}

// Hash keys [first, first+nk) of kd into h[PER] (key r*NT+t -> thread t, h[r]).
// `tile` is LDS scratch of K20Tile<NT, KPT>::kVec uint4 (K20 only).
#ifndef DLSM_TILE_ALL
#define DLSM_TILE_ALL 1  // hash_chunk: all key tiles of a chunk loaded at once (when they fit 16 uint4)
#endif
constexpr int kTileKPT = 2;  // keys per thread per LDS tile (20 KiB tiles at 512 threads)
// K28 (28-byte internal keys, ExtractUserKey = the first 20 bytes): the same
// LDS tiles at stride 7 dwords (odd: conflict-free), one key per thread per
// tile so a 1024-thread tile stays at 28 KiB (two persistent probe
// partition workgroups per CU).  The 8-byte trailers ride along in the
// coalesced 16-byte loads and are never hashed.
template <int MODE>
constexpr int mode_kb() { return MODE == KM_K28 ? 28 : 20; }
template <int KB>
constexpr int tile_kpt() { return KB == 20 ? kTileKPT : 1; }

// K20 with tiles 0 and 1 already in pre[0] / pre[1]: two key tiles stay in
// flight throughout -- while tile q is hashed, tile q+2 loads; while the last
// two tiles are hashed, the NEXT chunk's tiles 0 and 1 load (persistent loop:
// HBM reads continue through the bucket / scan / scatter / store phases).
template <int NT, int PER, int KB = 20>
__device__ __forceinline__ void hash_chunk_k20_pipe(const KeyDesc& kd, uint64_t first, uint32_t nk,
                                                    uint64_t next_first, uint32_t next_nk,
                                                    uint4* tile, uint32_t (&h)[PER],
                                                    uint4 (&pre)[2][K20Tile<NT, tile_kpt<KB>(), KB>::kPer]) {
  const int t = threadIdx.x;
  constexpr int KPT = tile_kpt<KB>();
  using TL = K20Tile<NT, KPT, KB>;
  constexpr int NTILES = PER / KPT;
  static_assert(NTILES >= 2, "two tiles in flight");
  const uint8_t* base = kd.bytes + first * KB;
  const uint8_t* nbase = kd.bytes + next_first * KB;
#pragma unroll
  for (int q = 0; q < NTILES; q++) {
    k20_tile_store<NT, KPT, KB>(tile, pre[q & 1]);
    __syncthreads();
    if (q + 2 < NTILES) {
      if ((q + 2) * TL::kKeys < static_cast<int>(nk)) k20_tile_fetch<NT, KPT, KB>(base, nk * KB, q + 2, pre[q & 1]);
    } else if (next_nk > static_cast<uint32_t>((q + 2 - NTILES) * TL::kKeys)) {
      k20_tile_fetch<NT, KPT, KB>(nbase, next_nk * KB, q + 2 - NTILES, pre[q & 1]);
    }
    const uint32_t* w = reinterpret_cast<const uint32_t*>(tile);
#pragma unroll
    for (int j = 0; j < KPT; j++) h[q * KPT + j] = hash_k20_lds(w + (KB / 4) * (j * NT + t));
    __syncthreads();
  }
}

template <int MODE, int NT, int PER>
__device__ __forceinline__ void hash_chunk(const KeyDesc& kd, uint64_t first, uint32_t nk,
                                           uint4* tile, uint32_t (&h)[PER]) {
  const int t = threadIdx.x;
  if constexpr (MODE == KM_K20 || MODE == KM_K28) {
    constexpr int KB = mode_kb<MODE>();
    constexpr int KPT = tile_kpt<KB>();
    using TL = K20Tile<NT, KPT, KB>;
    constexpr int NTILES = PER / KPT;
    const uint8_t* base = kd.bytes + first * KB;
    const uint32_t nbytes = nk * KB;
    if constexpr (DLSM_TILE_ALL && NTILES * TL::kPer <= 16) {
      // every tile's loads in flight at once (one HBM round trip per chunk,
      // not one per tile: short, non-persistent grids are latency-bound)
      uint4 all[NTILES][TL::kPer];
#pragma unroll
      for (int q = 0; q < NTILES; q++)
        if (q == 0 || q * TL::kKeys < static_cast<int>(nk)) k20_tile_fetch<NT, KPT, KB>(base, nbytes, q, all[q]);
#pragma unroll
      for (int q = 0; q < NTILES; q++) {
        k20_tile_store<NT, KPT, KB>(tile, all[q]);
        __syncthreads();
        const uint32_t* w = reinterpret_cast<const uint32_t*>(tile);
#pragma unroll
        for (int j = 0; j < KPT; j++) h[q * KPT + j] = hash_k20_lds(w + (KB / 4) * (j * NT + t));
        __syncthreads();
      }
      return;
    }
    uint4 pre[TL::kPer];
    k20_tile_fetch<NT, KPT, KB>(base, nbytes, 0, pre);
#pragma unroll
    for (int q = 0; q < NTILES; q++) {
      k20_tile_store<NT, KPT, KB>(tile, pre);
      __syncthreads();
      if (q + 1 < NTILES && (q + 1) * TL::kKeys < static_cast<int>(nk))
        k20_tile_fetch<NT, KPT, KB>(base, nbytes, q + 1, pre);
      const uint32_t* w = reinterpret_cast<const uint32_t*>(tile);
#pragma unroll
      for (int j = 0; j < KPT; j++) {
        const int r = q * KPT + j;
        h[r] = hash_k20_lds(w + (KB / 4) * (j * NT + t));
      }
      __syncthreads();
    }
  } else if constexpr (MODE == KM_HASH) {
    const uint32_t* hp = reinterpret_cast<const uint32_t*>(kd.bytes) + first;
#pragma unroll
    for (int r = 0; r < PER; r++) {
      const uint32_t i = r * NT + t;
      h[r] = i < nk ? __builtin_nontemporal_load(hp + i) : 0u;  // coalesced dwords
    }
  } else {
#pragma unroll
    for (int r = 0; r < PER; r++) {
      const uint32_t i = r * NT + t;
      h[r] = i < nk ? key_hash<KM_GENERIC>(kd, first + i) : 0u;
    }
  }
}

// Consecutive-distinct count of a chunk (AddKey, full_filter_block.cc:45-48):
// key i counts unless its hash equals key i-1's.  `prev0` is the hash of the
// key before the chunk, or ~h(key 0) for a job's first chunk (key 0 counts).
template <int NT, int PER>
__device__ __forceinline__ uint32_t chunk_distinct(const uint32_t (&h)[PER], uint32_t nk,
                                                   uint32_t prev0, uint32_t* lastw,
                                                   uint32_t* wsum) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  constexpr int NW = NT / 64;
  if (lane == 63) {
#pragma unroll
    for (int r = 0; r < PER; r++) lastw[r * NW + w] = h[r];
  }
  __syncthreads();
  uint32_t cnt = 0;
#pragma unroll
  for (int r = 0; r < PER; r++) {
    uint32_t p = __shfl_up(h[r], 1, 64);
    if (lane == 0) p = w > 0 ? lastw[r * NW + w - 1] : (r > 0 ? lastw[(r - 1) * NW + NW - 1] : prev0);
    const uint32_t i = r * NT + t;
    if (i < nk && h[r] != p) cnt++;
  }
  cnt = wave_sum(cnt);
  if (lane == 0) wsum[w] = cnt;
  __syncthreads();
  uint32_t tot = 0;
#pragma unroll
  for (int q = 0; q < NW; q++) tot += wsum[q];
  return tot;
}

// Inclusive add-scan over the wave in DPP: row_shr 1/2/4/8 inside each
// 16-lane row, then row_bcast:15 / row_bcast:31 across rows (lanes outside a
// step's source read 0; no LDS traffic).
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x111, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x112, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x114, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x118, 0xf, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x142, 0xa, 0xf, false));
  v += static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x143, 0xc, 0xf, false));
  return v;
}

constexpr uint32_t kWin = 64;  // entries per walk window (one per lane)

// s_waitcnt vmcnt(0), expcnt and lgkmcnt left at their maxima (gfx9 simm16:
// vmcnt [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8]).
constexpr int kWaitVmcnt0 = 0x0F70;

// The wave's index in its workgroup as a wave-uniform (SGPR) value: derived
// from threadIdx.x the compiler would treat it, and every walk counter built
// from it, as divergent (exec-mask loops, vmcnt(0) waits on prefetches).
__device__ __forceinline__ int wave_id() {
  return __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
}

// A wave-uniform 64-bit value moved to SGPRs (lets the compiler keep the
// segment-boundary loop scalar: s_ff1 / s_flbit instead of per-lane loops).
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(x)));
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(x >> 32)));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// Segment walk over one group of up to 64 chunks.  Lane l holds segment l:
// its flat start `excl` inside the group (wave prefix scan of the counts) and
// dv = l*CHUNK + off - excl, where off is the segment's offset inside chunk
// l's region, so flat entry e of segment l sits at in-group offset e + dv.
// `nz` is the wave mask of non-empty segments.  Lanes past T take the
// window's first entry, so every index stays inside the group.
// Located with LDS help, no per-boundary scalar loop.  At group setup the non-empty segments' dv are
// compacted into the wave's LDS list dvc[0..); per window, every segment
// that starts inside the window marks its start lane in the wave's 64-flag
// array, one ballot of the flags gives the window's boundary mask B, and lane
// j's segment is the (cw + popcount(B & lanes <= j))-th non-empty one, cw =
// the count of segments started at or before the window start.  Cost per
// window: 2 LDS writes + 2 LDS reads + 2 ballots + a few VALU, against a
// dependent readlane / s_ff1 chain per boundary (ablation: the walk alone
// took 87 of the slice pass's 177 us).  The arrays are wave-private and a
// wave's LDS operations complete in order, so no barrier is needed; a
// wavefront-scope fence between the flag stores and the flag load keeps the
// compiler from treating the exchange as single-thread memory.  The pointers
// carry the LDS address space (a generic pointer would become flat accesses).
constexpr int kWalkScratch = 192;  // u32 per wave: 64 x min(U, 2) flags + 64 compacted dv
typedef __attribute__((address_space(3))) uint32_t lds_u32;
// flags per wave for a walk of U windows per set (seg_locate_set_lds for U <= 2)
template <int U>
constexpr int walk_flags() { return U <= 2 ? 64 * U : 64; }

template <int U>
__device__ __forceinline__ void seg_locate_win_lds(uint32_t excl, uint64_t nz, uint32_t T, uint32_t w0,
                                                   lds_u32* flg, const lds_u32* dvc,
                                                   uint32_t (&idx)[U], bool (&ok)[U]) {
  const uint32_t lane = threadIdx.x & 63;
  const bool live = (nz >> lane) & 1u;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint32_t w = w0 + u * kWin;
    if (w >= T) {  // wave-uniform; never for u = 0 (next() only runs with e0 < T)
      ok[u] = false;
      idx[u] = u > 0 ? idx[0] : lane;  // re-reads window 0's units: see walk_segments
      continue;
    }
    const uint32_t cw = static_cast<uint32_t>(__builtin_popcountll(uniform64(__ballot(excl <= w) & nz)));
    flg[lane] = 0u;
    const uint32_t r = excl - w;
    if (live && excl > w && r < kWin) flg[r] = 1u;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const uint32_t f = flg[lane];
    const uint64_t b = __ballot(f != 0u);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(b >> 32),
                                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(b), 0u));
    const uint32_t d = dvc[cw + below + f - 1u];
    const uint32_t id = w + lane + d;
    const uint32_t id0 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(id), 0));
    ok[u] = w + lane < T;
    idx[u] = ok[u] ? id : id0;
  }
}

// Set-wide form (U <= 2): the flags of the whole window set
// are marked at once and stamped with the set's tag instead of being cleared
// (a wave-private running count, the array initialised to ~0 at the walk's
// start), so a set costs one flag store, one fence, then per window one flag
// read + one list read, and the windows' chains are independent.  A segment
// starting exactly at window u's start is counted in cw, so lane 0's flag is
// ignored.
template <int U>
__device__ __forceinline__ void seg_locate_set_lds(uint32_t excl, uint64_t nz, uint32_t T, uint32_t w0,
                                                   uint32_t tag, lds_u32* flg, const lds_u32* dvc,
                                                   uint32_t (&idx)[U], bool (&ok)[U]) {
  const uint32_t lane = threadIdx.x & 63;
  const bool live = (nz >> lane) & 1u;
  const uint32_t r = excl - w0;
  if (live && excl > w0 && r < kWin * U) flg[r] = tag;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // Branch-free over the set (the windows' LDS reads can overlap): a window
  // past T (u > 0 only: next() runs with w0 < T) is located anyway -- its list
  // index masked into the wave's scratch -- then replaced by window 0.
  uint32_t f[U];
#pragma unroll
  for (int u = 0; u < U; u++) f[u] = flg[u * kWin + lane];  // unconditional: no exec-masked reads
#pragma unroll
  for (int u = 0; u < U; u++) f[u] = (f[u] == tag) & (lane != 0u);
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint32_t w = w0 + u * kWin;
    const uint32_t cw = static_cast<uint32_t>(__builtin_popcountll(uniform64(__ballot(excl <= w) & nz)));
    const uint64_t b = __ballot(f[u] != 0u);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(b >> 32),
                                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(b), 0u));
    const uint32_t d = dvc[(cw + below + f[u] - 1u) & 63u];
    const uint32_t id = w + lane + d;
    const uint32_t id0 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(id), 0));
    const bool live_w = u == 0 || w < T;  // wave-uniform
    ok[u] = live_w && w + lane < T;
    idx[u] = ok[u] ? id : (live_w ? id0 : idx[0]);
  }
}

// One wave's walk over a slice's segments in the chunk groups g = g_first,
// g_first + g_step, ... < g_end (gs <= 64 chunks per group, one per lane: a
// caller with few chunks per wave shrinks gs so every wave of the workgroup
// gets a group instead of wave 0 walking them all; chunk-major table rows of
// `rowlen` u16 bucket offsets, `tb` already offset to the slice's column).
// Software-pipelined: window set i+1's hash loads (and the next group's table
// rows, one group ahead) are issued before window set i is consumed, so every
// wave keeps a set of loads in flight while it works on the previous one --
// the un-pipelined walk spent most of its cycles waiting on these loads.
// act(hv[U], idx[U], ok[U], g) consumes one window set of group g.
// E: the walk's element -- uint32_t (one entry) or uint4 (a 16-byte unit of
// four entries, for bucket offsets that are multiples of 4); CHUNK: a
// chunk region's stride in elements.
// NTL: the entry loads are non-temporal (the probe's 4 B/key entries are read
// once; streaming them past the Infinity Cache keeps it for the answers the
// unpermute pass reads next).
template <int U, uint32_t CHUNK, typename E = uint32_t, bool NTL = false>
struct SegWalk {
  static constexpr uint32_t kPerE = sizeof(E) / 4;  // entries per element
  const uint16_t* tb;
  const uint32_t* entries;
  uint32_t rowlen, g_step, g_end;
  uint32_t gs;        // chunks per group (<= 64; lanes >= gs hold empty segments)
  uint32_t g;         // current group (first chunk)
  uint32_t e0;        // next window start in the current group
  lds_u32* scr;       // the wave's kWalkScratch u32 of LDS
  uint32_t tag;       // window sets located so far (seg_locate_set_lds stamps)
  static constexpr int kFlags = walk_flags<U>();
  uint32_t excl, dv, T;
  uint64_t nz;        // non-empty segments of the current group
  uint32_t nrow;      // prefetched table row pair of group g + g_step (this lane's chunk), packed
  uint32_t chunk_rt;  // CHUNK == 0: the chunk region stride in elements, known at run time only
  __device__ __forceinline__ uint32_t stride() const { return CHUNK ? CHUNK : chunk_rt; }

  // The row pair (bucket start, bucket end) of this lane's chunk as one
  // packed u32, unpacked only in setup(): the load stays in flight until the
  // next group starts instead of being waited on where it is issued.
  __device__ __forceinline__ uint32_t load_rows(uint32_t gg) const {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c = min(min(gg, g_end) + lane, g_end - 1u);  // clamped: unconditional loads
    const uint16_t* r = tb + static_cast<uint64_t>(c) * rowlen;
    return static_cast<uint32_t>(r[0]) | (static_cast<uint32_t>(r[1]) << 16);
  }
  __device__ __forceinline__ void setup(uint32_t row) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t a0 = (row & 0xffffu) / kPerE, a1 = (row >> 16) / kPerE;
    const uint32_t cnt = lane < gs && g + lane < g_end ? a1 - a0 : 0u;
    const uint32_t incl = wave_incl_scan_dpp(cnt);
    excl = incl - cnt;
    T = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(incl), 63));
    dv = lane * stride() + a0 - excl;
    nz = uniform64(__ballot(cnt != 0u));
    e0 = 0;
    if (cnt != 0u) {  // compact the non-empty segments' dv (ordered by lane = by excl)
      const uint32_t k = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(nz >> 32),
                                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(nz), 0u));
      scr[kFlags + k] = dv;
    }
  }
  // The next group's rows are prefetched unconditionally (load_rows clamps
  // past-the-end groups to the last chunk): a prefetch under a branch makes
  // the compiler merge the two values of nrow with a copy that waits
  // (s_waitcnt vmcnt(0)) right after the load is issued.
  // begin() issues the first group's row loads (and the next group's) and
  // returns the first row pair without waiting for it; start() hands it to
  // setup().  A caller with a prologue of its own runs it in between, so the
  // row loads' round trip overlaps it.
  __device__ __forceinline__ bool begin(uint32_t g_first, uint32_t& row) {
    g = g_first;
    if (g >= g_end) return false;
    if constexpr (U <= 2) {
#pragma unroll
      for (int u = 0; u < kFlags / 64; u++) scr[u * 64 + (threadIdx.x & 63)] = ~0u;
      tag = 0;
    }
    row = load_rows(g);
    nrow = load_rows(g + g_step);
    return true;
  }
  __device__ __forceinline__ bool start(uint32_t g_first) {
    uint32_t row;
    if (!begin(g_first, row)) return false;
    setup(row);
    return true;
  }
  // Locate the next window set; false when the walk is done.
  __device__ __forceinline__ bool next(uint32_t (&idx)[U], bool (&ok)[U], uint32_t& gset) {
    if (e0 >= T) {
      g += g_step;
      if (g >= g_end) return false;
      setup(nrow);
      nrow = load_rows(g + g_step);  // after setup: the load can refill nrow's register (no copy, no wait)
      // Empty groups (rare): their successors' rows are loaded and waited
      // on here.  Reusing the prefetched row in this loop would put a use of
      // a just-issued load on one path into the group change, and the
      // compiler's single wait for nrow there would be a vmcnt(0) on every
      // path -- a drain of every load and store in flight once per group.
      while (e0 >= T) {
        g += g_step;
        if (g >= g_end) return false;
        const uint32_t row2 = load_rows(g);
        nrow = load_rows(g + g_step);
        setup(row2);
      }
    }
    if constexpr (U <= 2)
      seg_locate_set_lds<U>(excl, nz, T, e0, tag++, scr, scr + kFlags, idx, ok);
    else
      seg_locate_win_lds<U>(excl, nz, T, e0, scr, scr + kFlags, idx, ok);
    e0 += kWin * U;
    gset = g;
    return true;
  }
  __device__ __forceinline__ void fetch(const uint32_t (&idx)[U], uint32_t gset, E (&hv)[U]) const {
    const E* gent = reinterpret_cast<const E*>(entries) + static_cast<uint64_t>(gset) * stride();
#pragma unroll
    for (int u = 0; u < U; u++) {  // in-group for every lane: no select around the load
      if constexpr (NTL && sizeof(E) == 16) {
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(gent + idx[u]));
        hv[u] = make_uint4(x.x, x.y, x.z, x.w);
      } else {
        hv[u] = gent[idx[u]];
      }
    }
  }
};

// Window sets in flight per wave: set i+DEPTH's loads are issued before set i
// is consumed.  DEPTH 2 keeps two sets of loads in flight (the walk of a
// U = 1 unit window is short next to a loaded HBM round trip).
template <int U, uint32_t CHUNK, typename E>
struct WinSet {
  uint32_t idx[U], g;
  E hv[U];
  bool ok[U];
};

struct NoPrologue {
  __device__ __forceinline__ void operator()() const {}
};

// pro(): the caller's prologue (e.g. its slice image into LDS + a barrier),
// run by every wave after the first row loads are issued and before they are
// used -- their round trip overlaps it.  Every wave runs it, walk or not, so
// it may hold workgroup barriers.
template <int U, uint32_t CHUNK, typename E = uint32_t, int DEPTH = 1, bool NTL = false, typename Act,
          typename Pro = NoPrologue>
__device__ __forceinline__ void walk_segments(const uint16_t* tb, uint32_t rowlen, const uint32_t* entries,
                                              uint32_t g_first, uint32_t g_step, uint32_t g_end, uint32_t gs,
                                              uint32_t* scratch, Act act, Pro pro = Pro{},
                                              uint32_t chunk_rt = 0) {
  static_assert(DEPTH == 1 || DEPTH == 2, "walk depth");
  SegWalk<U, CHUNK, E, NTL> w{tb, entries, rowlen, g_step, g_end, gs};
  w.chunk_rt = chunk_rt;
  w.scr = (lds_u32*)scratch;  // generic -> LDS address space (addrspacecast)
  uint32_t row0 = 0;
  const bool any = w.begin(g_first, row0);
  pro();
  if (!any) return;
  w.setup(row0);
  WinSet<U, CHUNK, E> A, B;
  if (!w.next(A.idx, A.ok, A.g)) return;
  w.fetch(A.idx, A.g, A.hv);
  // The first set's loads land in A's registers, which the loop refills by
  // copies: left pending into the loop, the compiler's wait for them merges
  // with the loop's state into an s_waitcnt vmcnt(0) placed right after every
  // iteration's prefetch -- each set's loads were waited on where they were
  // issued.  Waiting once here keeps the loop's waits at the copies.
  __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
  bool haveB = false;
  if constexpr (DEPTH == 2) {
    haveB = w.next(B.idx, B.ok, B.g);
    if (haveB) w.fetch(B.idx, B.g, B.hv);
  }
  while (true) {
    WinSet<U, CHUNK, E> N;
    const bool more = (DEPTH == 1 || haveB) && w.next(N.idx, N.ok, N.g);
    if (more) w.fetch(N.idx, N.g, N.hv);
    act(A.hv, A.idx, A.ok, A.g);
    if constexpr (DEPTH == 1) {
      if (!more) break;
      A = N;
    } else {
      if (!haveB) break;
      A = B;
      B = N;
      haveB = more;
    }
  }
}

// Copy n u32 / u16 staged in LDS to global memory with 16-byte stores (the
// global base is 16-byte aligned: chunk starts are multiples of 4096 elements).
// NTS: non-temporal 16-byte stores.  The probe's intermediates (≈520 MB per
// 100 M keys) cannot stay in the 256 MiB Infinity Cache anyway, so streaming
// them past it keeps it for the key stream (probe: −5 %); the build's 4 B/key
// hashes do fit and are re-read by the slice pass, so the build keeps plain
// stores.
template <bool NTS>
__device__ __forceinline__ void store16(uint4* g, const uint4& v) {
  if constexpr (NTS) {
    u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(g));
  } else {
    *g = v;
  }
}
template <int NT, bool NTS = false>
__device__ __forceinline__ void store_chunk_u32(uint32_t* g, const uint32_t* lds, uint32_t n) {
  const uint32_t nv = n / 4u;
  for (uint32_t v = threadIdx.x; v < nv; v += NT)
    store16<NTS>(reinterpret_cast<uint4*>(g) + v, reinterpret_cast<const uint4*>(lds)[v]);
  for (uint32_t i = nv * 4u + threadIdx.x; i < n; i += NT) g[i] = lds[i];
}
template <int NT, bool NTS = false>
__device__ __forceinline__ void store_chunk_u16(uint16_t* g, const uint16_t* lds, uint32_t n) {
  const uint32_t nv = n / 8u;
  for (uint32_t v = threadIdx.x; v < nv; v += NT)
    store16<NTS>(reinterpret_cast<uint4*>(g) + v, reinterpret_cast<const uint4*>(lds)[v]);
  for (uint32_t i = nv * 8u + threadIdx.x; i < n; i += NT) g[i] = lds[i];
}

// ---------------------------------------------------------------------------
// Full filter build, pass 1: hash + consecutive-dedup count (+ slice
// partition).  One 512-thread workgroup per chunk of kBuildChunk keys of one
// job.
// ---------------------------------------------------------------------------
// Build entries: AddHash reads only hash bits
// [0, 9) and [17, 26) (bitpos = h & 511 stepping by rotr(h, 17), positions
// mod 512, util/bloom_impl.h:427-443), so the partition parks the key's line
// offset inside its slice (< 2^11) in bits [9, 17) and [26, 29): the slice
// pass needs no modulo.  The full hash is gone, so the rare slice fallback
// (duplicates lowered L) re-hashes the keys.
// Bit 31 is never read either: real entries clear it, bucket padding sets it.
[[maybe_unused]] constexpr uint32_t kBuildPadEntry = 0x80000000u;
__device__ __forceinline__ uint32_t build_entry(uint32_t h, uint32_t off) {
  return (h & 0x63FE01FFu) | ((off & 0xffu) << 9) | ((off >> 8) << 26);
}
__device__ __forceinline__ uint32_t build_entry_off(uint32_t e) {
  return ((e >> 9) & 0xffu) | (((e >> 26) & 7u) << 8);
}

constexpr int kPartBlock = kBuildChunk / 8;  // 8 keys per thread (512 threads at 4,096-key chunks)

// Job-wide distinct count (defined below; used by the exact partition).
template <int NT>
__device__ __forceinline__ uint64_t job_distinct(const FullJobDev& J, const uint32_t* dchunk,
                                                 uint32_t* wsum64);

// EXACT (PART only): the count pass already wrote every chunk's distinct count
// to dchunk, so each workgroup sums its job's counts and buckets by the true
// line count instead of the speculative one.
template <int MODE, bool PART, bool EXACT = false>
__global__ __launch_bounds__(kPartBlock) void full_partition_kernel(
    const FullJobDev* __restrict__ jobs, const uint32_t* __restrict__ chunk0s, int n_jobs,
    uint32_t* __restrict__ dchunk, uint32_t* __restrict__ entries, uint16_t* __restrict__ tab,
    int lgR, uint32_t block0) {
  constexpr int C = kBuildChunk;
  constexpr int PER = C / kPartBlock;
  // key tile (K20), then the staging area of the bucketed hashes (both modes)
  constexpr int KB = mode_kb<MODE>();
  constexpr int TKV = K20Tile<kPartBlock, tile_kpt<KB>(), KB>::kVec;
  constexpr int RV = static_cast<int>(kBuildRegion) / 4;  // the staging area holds a (padded) chunk
  constexpr int TVB = TKV > RV ? TKV : RV;
  __shared__ __attribute__((aligned(16))) uint4 tile[TVB];
  __shared__ uint32_t hist[kMaxSlices + 1];
  __shared__ uint8_t npad[kMaxSlices + 1];
  __shared__ uint32_t lastw[PER * (kPartBlock / 64)];
  __shared__ uint32_t wsum[kPartBlock / 64];
  __shared__ int sj;
  const int tid = threadIdx.x;
  const uint32_t bid = blockIdx.x + block0;  // chunk index over all jobs
  if (tid == 0) sj = find_job(chunk0s, n_jobs, bid);
  __syncthreads();
  const FullJobDev J = jobs[sj];
  const uint32_t c = bid - J.chunk0;
  const uint64_t first = static_cast<uint64_t>(c) * C;
  const uint64_t left = J.keys.n - first;
  const uint32_t nk = left < static_cast<uint64_t>(C) ? static_cast<uint32_t>(left) : C;

  // the key before the chunk (AddKey's dedup neighbour), hashed before the
  // chunk's tile loads so its round trip overlaps them
  uint32_t prev_h = 0;
  if (!EXACT && first > 0 && tid == 0) prev_h = key_hash<MODE>(J.keys, first - 1);  // only wave 0 lane 0 reads it
  uint32_t h[PER];
  hash_chunk<MODE, kPartBlock, PER>(J.keys, first, nk, tile, h);
  uint32_t L = J.L_spec, magic = J.magic_spec;
  if constexpr (EXACT) {
    L = full_num_lines(job_distinct<kPartBlock>(J, dchunk, wsum), J.bpk, nullptr);
    magic = fastmod_magic(L);
  } else {
    const uint32_t prev0 = first > 0 ? __shfl(prev_h, 0, 64) : ~__shfl(h[0], 0, 64);
    const uint32_t cnt = chunk_distinct<kPartBlock, PER>(h, nk, prev0, lastw, wsum);
    if (tid == 0) dchunk[bid] = cnt;
  }
  if constexpr (!PART) return;

  const uint32_t S = J.n_slices;
  for (uint32_t b = tid; b <= S; b += kPartBlock) hist[b] = 0;
  __syncthreads();
  uint32_t code[PER];
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const uint32_t i = r * kPartBlock + tid;
    if (i < nk) {
      const uint32_t line = fastmod(h[r], L, magic);
      const uint32_t s = line >> lgR;
      code[r] = (atomicAdd(&hist[s], 1u) << 9) | s;
      h[r] = build_entry(h[r], line & ((1u << lgR) - 1u));
    }
  }
  __syncthreads();
  for (uint32_t b = tid; b < S; b += kPartBlock) {  // pad every bucket to whole 16-byte units
    const uint32_t pad = (0u - hist[b]) & 3u;
    npad[b] = static_cast<uint8_t>(pad);
    hist[b] += pad;
  }
  __syncthreads();
  const uint32_t total = block_excl_scan_lds<kPartBlock>(hist, static_cast<int>(S + 1), wsum);
  for (uint32_t b = tid; b <= S; b += kPartBlock)
    tab[J.tab0 + static_cast<uint64_t>(c) * (S + 1) + b] = static_cast<uint16_t>(hist[b]);
  uint32_t* stage = reinterpret_cast<uint32_t*>(tile);  // free since hash_chunk's last barrier
  for (uint32_t b = tid; b < S; b += kPartBlock) {
    const uint32_t end = hist[b + 1], np = npad[b];
    if (np > 0) stage[end - 1] = kBuildPadEntry;
    if (np > 1) stage[end - 2] = kBuildPadEntry;
    if (np > 2) stage[end - 3] = kBuildPadEntry;
  }
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const uint32_t i = r * kPartBlock + tid;
    if (i < nk) stage[hist[code[r] & 511u] + (code[r] >> 9)] = h[r];
  }
  __syncthreads();
  store_chunk_u32<kPartBlock>(entries + J.entry0 + static_cast<uint64_t>(c) * kBuildRegion, stage, total);
}

// Sum of a job's per-chunk distinct counts (every thread gets the total).
template <int NT>
__device__ __forceinline__ uint64_t job_distinct(const FullJobDev& J, const uint32_t* dchunk,
                                                 uint32_t* wsum64) {
  __syncthreads();  // wsum64 may still be read from a previous use
  uint32_t lo = 0;
  for (uint32_t c = threadIdx.x; c < J.n_chunks; c += NT) lo += dchunk[J.chunk0 + c];
  // chunk counts are <= 4096, so a 32-bit partial per thread cannot overflow
  // for < 2^20 chunks per thread; sum in 64 bits across threads
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t ws = wave_sum(lo);
  if (lane == 0) wsum64[w] = ws;
  __syncthreads();
  uint64_t tot = 0;
#pragma unroll
  for (int q = 0; q < NT / 64; q++) tot += wsum64[q];
  __syncthreads();
  return tot;
}

// ---------------------------------------------------------------------------
// Full filter build, pass 2 (sliced): one 512-thread workgroup per (job, slice
// of 2^LGR lines).  The slice lives in LDS; each wave walks the slice's
// segments of 64 chunks at a time (wave prefix scan + ds_bpermute search, 4
// entries in flight per lane), ORs bits with ds_or, and the slice streams out
// with 16-byte stores.
// ---------------------------------------------------------------------------
constexpr int kSliceBlock = 512;

// ---- crc32c of a filter slice (sealed blocks, round 6) --------------------
// Reflected Castagnoli arithmetic as in block_crc.hip: the register after
// bytes A||B is reg(A) * x^(8|B|) xor raw(B) (raw: the register run from 0),
// and leading zero bytes leave a zero register unchanged.  A slice of nl
// lines (nl * 64 bytes) is front-padded with zeros to R * 64 bytes; thread t
// runs the table CRC over its 16 * R / 512 words (the filter's first byte
// seeds the register with 0xffffffff, crc32c's initial value), and its
// register, times x^(8 * bytes after its segment) from a host table, is
// XOR-reduced over the workgroup.
__device__ __forceinline__ uint32_t crc_mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    p ^= (a & (0x80000000u >> i)) ? b : 0u;
    b = (b >> 1) ^ ((b & 1u) ? 0x82f63b78u : 0u);
  }
  return p;
}
#ifndef DLSM_CRC_NIB
#define DLSM_CRC_NIB 1  // slice CRC by 4-bit tables (8 conflict-free lookups / word) instead of byte tables
#endif
__device__ __forceinline__ uint32_t crc_word(uint32_t r, uint32_t w, const uint32_t* T) {
  r ^= w;
  if constexpr (DLSM_CRC_NIB) {
    // T: 8 tables of 16 (nibble q of the register): 16 entries in 16 banks,
    // so a lookup instruction never conflicts (random byte tables: ~3.5-way)
    uint32_t x = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) x ^= T[16 * q + ((r >> (4 * q)) & 15u)];
    return x;
  } else {
    return T[768 + (r & 0xffu)] ^ T[512 + ((r >> 8) & 0xffu)] ^ T[256 + ((r >> 16) & 0xffu)] ^ T[r >> 24];
  }
}
template <uint32_t R>
__device__ __forceinline__ uint32_t crc_slice_partial(const uint32_t* sl, uint32_t nl, bool seed,
                                                      const uint32_t* T, uint32_t shift, uint32_t* wsum) {
  constexpr uint32_t WPT = R * 16u / kSliceBlock;  // words per thread (multiple of 4: R >= 128)
  static_assert(WPT % 4 == 0, "whole 16-byte reads");
  const uint32_t tid = threadIdx.x;
  const uint32_t padw = (R - nl) * 16u;  // zero words in front (a multiple of 16)
  uint32_t r = 0;
#pragma unroll
  for (uint32_t q = 0; q < WPT / 4; q++) {
    const uint32_t i = tid * WPT + 4u * q;  // first word of this 16-byte piece (padded numbering)
    if (i >= padw) {
      const uint4 v = *reinterpret_cast<const uint4*>(sl + (i - padw));
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
      if (seed && i == padw) r = 0xffffffffu;  // the filter's first byte: crc32c's initial register
#pragma unroll
      for (int j = 0; j < 4; j++) r = crc_word(r, w4[j], T);
    }
  }
  r = crc_mulmod(r, shift);  // x^(8 * WPT * 4 * (threads after this one)), loaded at kernel start
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) r ^= __shfl_xor(r, d, 64);
  __syncthreads();  // wsum is free (the walk and job_distinct are done)
  if ((tid & 63) == 0) wsum[tid >> 6] = r;
  __syncthreads();
  uint32_t t = 0;
#pragma unroll
  for (int w = 0; w < kSliceBlock / 64; w++) t ^= wsum[w];
  return t;
}

#ifndef DLSM_SEAL_LAST
#define DLSM_SEAL_LAST 0  // 1: the last slice workgroup of a job seals it (0: a seal kernel launch)
#endif
// The crc32c register after a filter's L lines from its slices' partials
// (slice s's register times x^(8 * bytes of the slices after it): P1 for
// whole slices, P64 for the last slice's lines); the workgroup's threads fold
// a slice each.  Partials are read with agent-scope loads (other XCDs wrote
// them).  The result is meaningful in thread 0.
template <uint32_t R>
__device__ __forceinline__ uint32_t crc_seal_fold(const uint32_t* part, uint32_t L, const uint32_t* crc_tabs,
                                                  uint32_t* wsum) {
  const uint32_t S = (L + R - 1u) / R;  // slices holding bytes
  const uint32_t* P1 = crc_tabs + 1024 + kSliceBlock;
  const uint32_t* P64 = P1 + 256;
  uint32_t x = 0;
  for (uint32_t t = threadIdx.x; t + 1u < S; t += kSliceBlock)
    x ^= crc_mulmod(__hip_atomic_load(part + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), P1[S - 2u - t]);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x ^= __shfl_xor(x, d, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x != 0) return 0;
  x = 0;
#pragma unroll
  for (int w = 0; w < kSliceBlock / 64; w++) x ^= wsum[w];
  if (S == 0) return 0xffffffffu;  // no lines: the trailer's first byte starts the crc
  return crc_mulmod(x, P64[L - (S - 1u) * R]) ^
         __hip_atomic_load(part + (S - 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Run the register through the trailer (k, Fixed32 L) and the type byte (0);
// append [type 0][crc32c::Mask(value)] at `t` (table/table_builder_computeside.cc:418-428).
__device__ __forceinline__ void crc_seal_append(uint8_t* t, uint32_t r, uint32_t L, int k) {
  const uint8_t tail[6] = {static_cast<uint8_t>(static_cast<int8_t>(k)), static_cast<uint8_t>(L),
                           static_cast<uint8_t>(L >> 8), static_cast<uint8_t>(L >> 16),
                           static_cast<uint8_t>(L >> 24), 0u};
  // bit by bit: six table lookups would be six dependent global loads
#pragma unroll
  for (int b = 0; b < 6; b++) {
    r ^= tail[b];
#pragma unroll
    for (int i = 0; i < 8; i++) r = (r >> 1) ^ (0x82f63b78u & (0u - (r & 1u)));
  }
  const uint32_t value = ~r;
  const uint32_t m = ((value >> 15) | (value << 17)) + 0xa282ead8u;  // crc32c::Mask
  t[0] = 0;  // kNoCompression
  t[1] = static_cast<uint8_t>(m);
  t[2] = static_cast<uint8_t>(m >> 8);
  t[3] = static_cast<uint8_t>(m >> 16);
  t[4] = static_cast<uint8_t>(m >> 24);
}        // build slices (32 KiB LDS -> 4 per CU)
// probe slices: 64 KiB LDS per workgroup, 512 or 1024 threads (launch_probe_slices)
#ifndef DLSM_BUILD_WALKU
#define DLSM_BUILD_WALKU 8
#endif
#ifndef DLSM_BUILD_DEPTH
#define DLSM_BUILD_DEPTH 1  // window sets of entry loads in flight per wave (build walk)
#endif
#ifndef DLSM_BUILD_GS
#define DLSM_BUILD_GS 0     // chunks per wave group for jobs of >= 256 chunks (0: 64)
#endif
constexpr int kWalkU = DLSM_BUILD_WALKU;  // hashes in flight per lane (build segment walk)
#ifndef DLSM_PROBE_U
#define DLSM_PROBE_U 1
#endif
#ifndef DLSM_PROBE_NTL
#define DLSM_PROBE_NTL 1  // non-temporal entry loads in the probe slice pass
#endif
#ifndef DLSM_PROBE_DEPTH
#define DLSM_PROBE_DEPTH 1  // window sets of loads in flight per wave (walk_segments)
#endif
#ifndef DLSM_PROBE_NT
#define DLSM_PROBE_NT 1024  // probe slice workgroup size (two 64 KiB slices per CU)
#endif
#ifndef DLSM_PROBE_MINWAVES
#define DLSM_PROBE_MINWAVES 1
#endif
#ifndef DLSM_PROBE_U8
#define DLSM_PROBE_U8 2
#endif
constexpr int kProbeWalkU = DLSM_PROBE_U;    // probe walk, 64 KiB slices: unit windows in flight per wave
constexpr int kProbeWalkU8 = DLSM_PROBE_U8;  // probe walk, 128 KiB slices

// Publish a slice's crc partial at agent scope and count the slice in its
// job's counter (thread 0); *last = 1 in the workgroup whose count completes
// the job.  The caller's next barrier makes *last visible.
[[maybe_unused]] __device__ __forceinline__ void publish_slice_crc(uint32_t* part_slot, uint32_t part, uint32_t* cnt,
                                                  uint32_t n_slices, uint32_t* last) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(part_slot, part, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    *last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u == n_slices ? 1u : 0u;
  }
}

// CRC: the sealed filter block: once its lines
// are in LDS, the slice also computes the crc32c register contribution of its
// bytes (crc_slice_partial) into crc_part[slice]; full_block_seal_kernel folds
// a filter's partials, runs them through the trailer and the type byte, and
// appends [type 0][masked crc] -- no second pass over the filter bytes.
// Measured (profiles/r06_block_seal_ab.txt): the slice pass 50 -> 65-69 us
// for the bench's 16 x 2 MB filters plus a 5 us seal launch; sealing in the
// last slice workgroup of each filter instead (DLSM_SEAL_LAST=1: agent-scope
// partials, a release fence and a counter) costs more, 85-93 us, the fences.
template <int LGR, bool CRC = false>
__global__ __launch_bounds__(kSliceBlock) void full_slice_kernel(
    const FullJobDev* __restrict__ jobs, const uint32_t* __restrict__ slice0s, int n_jobs,
    const uint32_t* __restrict__ dchunk, const uint32_t* __restrict__ entries,
    const uint16_t* __restrict__ tab, uint32_t block0, uint32_t* __restrict__ crc_part = nullptr,
    const uint32_t* __restrict__ crc_tabs = nullptr, uint32_t* __restrict__ crc_cnt = nullptr) {
  constexpr uint32_t R = 1u << LGR;
  constexpr int NW = kSliceBlock / 64;
  __shared__ __attribute__((aligned(16))) uint32_t sl[R * 16];
  __shared__ uint32_t wsum[NW];
  __shared__ uint32_t walk_scr[NW * kWalkScratch];
  // crc32c tables (nibble: 512 B; 4 KiB more LDS would cost a workgroup per CU)
  __shared__ uint32_t crcT[CRC ? (DLSM_CRC_NIB ? 128 : 1024) : 1];
  __shared__ int sj;
  __shared__ uint32_t s_last;  // CRC: this workgroup completed its job's slice count
  const int tid = threadIdx.x;
  const int wv = wave_id();  // wave-uniform (SGPR): keeps the segment walk's control flow scalar
  const uint32_t bid = xcd_block(blockIdx.x, gridDim.x) + block0;  // slice index over all jobs
  if (tid == 0) sj = find_job(slice0s, n_jobs, bid);
  // CRC: this thread's shift multiplier, loaded beside the tables and waited
  // for before the first barrier, so that no wait for it after the filter
  // stores also waits for those stores (vmcnt counts loads and stores in order)
  uint32_t crc_shift = 0;
  if constexpr (CRC) crc_shift = crc_tabs[1024 + kSliceBlock - 1 - tid];
  for (uint32_t w = tid; w < R * 16; w += kSliceBlock) sl[w] = 0;
  if constexpr (CRC) {
    if constexpr (DLSM_CRC_NIB) {
      // nibble table q (byte q / 2 of the register, low or high half) from
      // the byte table the slice-by-4 step uses for that byte (linear in it)
      if (tid < 128u) {
        const uint32_t q = tid >> 4, v = tid & 15u;
        crcT[tid] = crc_tabs[(3u - (q >> 1)) * 256u + (v << (4u * (q & 1u)))];
      }
    } else {
      for (uint32_t w = tid; w < 1024u; w += kSliceBlock) crcT[w] = crc_tabs[w];
    }
    asm volatile("" : "+v"(crc_shift));
  }
  __syncthreads();
  const FullJobDev J = jobs[sj];
  const uint32_t s = bid - J.slice0;
  const uint64_t distinct = job_distinct<kSliceBlock>(J, dchunk, wsum);
  uint32_t total_bits;
  const uint32_t L = full_num_lines(distinct, J.bpk, &total_bits);
  const uint64_t len = static_cast<uint64_t>(total_bits / 8u) + 5u;
  if (len > J.out_cap) {
    if (s == 0 && tid == 0) *J.out_len = 0;
    return;
  }
  const uint32_t lo_line = s << LGR;
  uint32_t part = 0;  // CRC: this slice's register contribution (0: no bytes past a lowered L)
  if (L != 0 && lo_line < L) {
    const uint32_t magic = fastmod_magic(L);
    if (L == J.L_spec || J.exact) {  // the partition bucketed by this L
      const uint32_t nC = J.n_chunks;
      const uint16_t* tb = tab + J.tab0 + s;  // chunk-major rows of n_slices+1 u16
      const uint32_t* ent = entries + J.entry0;
      const int k = J.k;
      // chunks per wave group: every wave gets a share of a small job's chunks
      // (a job of >= 256 chunks keeps whole 64-chunk groups: measured 2 %
      // faster at 391 chunks than 8 groups of 49, gpurun_out v19b)
      const uint32_t gs = nC >= 256u ? (DLSM_BUILD_GS ? min(64u, max(1u, (nC + NW - 1) / NW))
                                                        : 64u)
                                     : max(1u, (nC + NW - 1) / NW);
      // 16-byte units of 4 entries per lane per load (padding entries skipped)
      constexpr int U4 = kWalkU / 4;
      walk_segments<U4, kBuildRegion / 4, uint4, DLSM_BUILD_DEPTH>(
          tb, J.n_slices + 1, ent, wv * gs, NW * gs, nC, gs, walk_scr + wv * kWalkScratch,
          [&](const uint4 (&hv)[U4], const uint32_t (&)[U4], const bool (&ok)[U4], uint32_t) {
            if (k == 6) {  // bits_per_key 10 (ChooseNumProbes): straight-line probes
#pragma unroll
              for (int u = 0; u < U4; u++) {
                const uint32_t e4[4] = {hv[u].x, hv[u].y, hv[u].z, hv[u].w};
#pragma unroll
                for (int j = 0; j < 4; j++)
                  if (ok[u] && !(e4[j] & kBuildPadEntry)) lds_add_hash_k<6>(sl + build_entry_off(e4[j]) * 16u, e4[j]);
              }
            } else {
#pragma unroll
              for (int u = 0; u < U4; u++) {
                const uint32_t e4[4] = {hv[u].x, hv[u].y, hv[u].z, hv[u].w};
#pragma unroll
                for (int j = 0; j < 4; j++)
                  if (ok[u] && !(e4[j] & kBuildPadEntry)) lds_add_hash(sl + build_entry_off(e4[j]) * 16u, e4[j], k);
              }
            }
          });
    } else {
      // Duplicates lowered the line count below the speculative one: the
      // partition used the wrong modulus (and the entries no longer hold the
      // full hash), so re-hash every key of the job.
      for (uint64_t e = tid; e < J.keys.n; e += kSliceBlock) {
        const uint32_t hv = key_hash<KM_GENERIC>(J.keys, e);
        const uint32_t line = fastmod(hv, L, magic);
        if ((line >> LGR) == s) lds_add_hash(sl + (line - lo_line) * 16u, hv, J.k);
      }
    }
    __syncthreads();
    const uint32_t nl = min(R, L - lo_line);
    // CRC + DLSM_SEAL_LAST: the partial is published before the filter
    // stores, so that the release fence does not wait for them to drain
    constexpr bool early = CRC && DLSM_SEAL_LAST;
    if constexpr (early) part = crc_slice_partial<R>(sl, nl, s == 0, crcT, crc_shift, wsum);
    if constexpr (early) publish_slice_crc(crc_part + bid, part, crc_cnt + sj, J.n_slices, &s_last);
    uint4* dst = reinterpret_cast<uint4*>(J.out + static_cast<uint64_t>(lo_line) * 64u);
    const uint4* src = reinterpret_cast<const uint4*>(sl);
    for (uint32_t w = tid; w < nl * 4u; w += kSliceBlock) st_global16(dst + w, src[w]);
    if constexpr (CRC && !early) part = crc_slice_partial<R>(sl, nl, s == 0, crcT, crc_shift, wsum);
  } else if constexpr (CRC && DLSM_SEAL_LAST) {
    publish_slice_crc(crc_part + bid, 0u, crc_cnt + sj, J.n_slices, &s_last);  // no bytes past a lowered L
  }
  if constexpr (CRC) {
#if DLSM_SEAL_LAST
    // The job's last slice workgroup to finish seals the filter (no seal
    // launch): every slice publishes its partial at agent scope, then counts
    // itself in the job's counter (publish_slice_crc, before its filter
    // stores); the one that completes the count reads the partials back
    // (agent-scope loads after an acquire fence), writes the trailer, the
    // block trailer and the length, and resets the counter for the next call.
    // Only the sealer writes the trailer bytes and out_len.
    __syncthreads();
    if (s_last) {
      __threadfence();
      const uint32_t r = crc_seal_fold<R>(crc_part + J.slice0, L, crc_tabs, wsum);
      if (tid == 0) {
        write_trailer(J.out, L, J.k);
        crc_seal_append(J.out + len, r, L, J.k);
        *J.out_len = len + 5u;
        crc_cnt[sj] = 0;
      }
    }
    return;
#else
    if (tid == 0) crc_part[bid] = part;
#endif
  }
  if (s == 0 && tid == 0) {
    write_trailer(J.out, L, J.k);
    *J.out_len = len;
  }
}

// Seal every filter of a sliced batch build (CRC slices): one workgroup per
// job folds its slices' partials -- slice s's register times x^(8 * bytes of
// the slices after it) from the host tables (P1: whole slices, P64: whole
// lines of the last slice) -- then runs the register through the 5-byte
// trailer and the type byte (0), and appends [type][crc32c::Mask(value)]
// (table/table_builder_computeside.cc:418-428): out_len += 5.  A job whose
// build failed (out_len 0) is left alone.
template <int LGR>
__global__ __launch_bounds__(256) void full_block_seal_kernel(const FullJobDev* __restrict__ jobs,
                                                              const uint32_t* __restrict__ crc_part,
                                                              const uint32_t* __restrict__ crc_tabs) {
  constexpr uint32_t R = 1u << LGR;
  __shared__ uint32_t wx[4];
  const FullJobDev J = jobs[blockIdx.x];
  const uint64_t len = *J.out_len;  // L * 64 + 5 (slice 0 wrote it), or 0
  if (len == 0) return;
  const uint32_t L = static_cast<uint32_t>((len - 5u) / 64u);
  const uint32_t S = (L + R - 1u) / R;  // slices holding bytes (a lowered L uses fewer)
  const uint32_t* P1 = crc_tabs + 1024 + kSliceBlock;  // x^(8 * R * 64 * m)
  const uint32_t* P64 = P1 + 256;                     // x^(8 * 64 * m)
  const uint32_t* part = crc_part + J.slice0;
  // thread 0's last-slice operands, loaded beside the other threads' partials
  uint32_t p_last = 0, last_part = 0;
  if (threadIdx.x == 0 && S != 0) {
    p_last = P64[L - (S - 1u) * R];
    last_part = part[S - 1u];
  }
  uint32_t x = 0;  // slices 0 .. S-2, each shifted to the end of slice S-2
  for (uint32_t t = threadIdx.x; t + 1u < S; t += 256u) x ^= crc_mulmod(part[t], P1[S - 2u - t]);
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) x ^= __shfl_xor(x, d, 64);
  if ((threadIdx.x & 63) == 0) wx[threadIdx.x >> 6] = x;
  __syncthreads();
  if (threadIdx.x != 0) return;
  x = wx[0] ^ wx[1] ^ wx[2] ^ wx[3];
  uint32_t r = 0xffffffffu;  // no lines (an empty filter): the trailer's first byte starts the crc
  if (S != 0) r = crc_mulmod(x, p_last) ^ last_part;  // after the last slice's lines
  crc_seal_append(J.out + len, r, L, J.k);
  *J.out_len = len + 5u;
}

// ---------------------------------------------------------------------------
// Full filter build, direct path: count -> zero + trailer -> global-atomic
// scatter.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void full_zero_kernel(const FullJobDev* __restrict__ jobs,
                                                           const uint32_t* __restrict__ dchunk,
                                                           uint32_t* __restrict__ jobL) {
  __shared__ uint32_t wsum[kBlock / 64];
  const FullJobDev J = jobs[blockIdx.y];
  const uint64_t distinct = job_distinct<kBlock>(J, dchunk, wsum);
  uint32_t total_bits;
  const uint32_t L = full_num_lines(distinct, J.bpk, &total_bits);
  const uint64_t len = static_cast<uint64_t>(total_bits / 8u) + 5u;
  if (len > J.out_cap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      *J.out_len = 0;
      jobL[blockIdx.y] = 0xffffffffu;
    }
    return;
  }
  uint4* o = reinterpret_cast<uint4*>(J.out);
  const uint64_t vecs = static_cast<uint64_t>(L) * 4u;
  for (uint64_t w = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x; w < vecs;
       w += static_cast<uint64_t>(gridDim.x) * kBlock)
    o[w] = make_uint4(0, 0, 0, 0);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    write_trailer(J.out, L, J.k);
    *J.out_len = len;
    jobL[blockIdx.y] = L;
  }
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void full_scatter_kernel(
    const FullJobDev* __restrict__ jobs, const uint32_t* __restrict__ chunk0s, int n_jobs,
    const uint32_t* __restrict__ jobL) {
  __shared__ int sj;
  if (threadIdx.x == 0) sj = find_job(chunk0s, n_jobs, static_cast<uint32_t>(blockIdx.x));
  __syncthreads();
  const int j = sj;
  const uint32_t L = jobL[j];
  if (L == 0 || L == 0xffffffffu) return;
  const FullJobDev J = jobs[j];
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
    const uint32_t h = key_hash<(MODE == KM_K20 || MODE == KM_HASH) ? MODE : KM_GENERIC>(kd, i);
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
// Bit-transposed stacked image: byte (line*512 + bit) holds bit `bit` of line
// `line` of filter f in its bit f, so one 1-byte LDS read answers a probe for
// all 8 filters and ANDing the k bytes gives the key's answer byte directly.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void stack_filters_kernel(const FilterDev* __restrict__ slots,
                                                               uint64_t words,
                                                               uint64_t* __restrict__ stacked) {
  __shared__ const uint8_t* src[8];
  if (threadIdx.x < 8) src[threadIdx.x] = slots[threadIdx.x].data;
  __syncthreads();
  for (uint64_t w = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x; w < words;
       w += static_cast<uint64_t>(gridDim.x) * kBlock) {
    uint64_t x = 0;  // byte b = byte w of the filter in slot b (0 for an empty slot)
#pragma unroll
    for (int f = 0; f < 8; f++)
      if (src[f]) x |= static_cast<uint64_t>(src[f][w]) << (8 * f);
    // 8x8 bit transpose: bit b of byte f -> bit f of byte b
    uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
    x ^= t ^ (t << 7);
    t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
    x ^= t ^ (t << 14);
    t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
    x ^= t ^ (t << 28);
    stacked[w] = x;  // bytes w*8 .. w*8+7 = bit positions 8*(w%64) .. +7 of line w/64
  }
}

// A probe only reads hash bits [0, 9) (first bit position) and [17, 26)
// (the low 9 bits of delta = rotr(h, 17)): HashMayMatchPrepared,
// util/bloom_impl.h:466-479, with every position taken mod 512.  The
// partition therefore parks the key's line offset inside its slice (< 256)
// in the unused bits [9, 17), so the slice pass needs no modulo: the LDS base
// of the key's line is `e & kEntryLineMask` (= offset * 512) and the
// positions are (e + q * (e >> 17)) & 511, exactly those of h.
// Bit 31 is never read either: valid entries clear it, and the bucket
// padding is kProbePadEntry (bit 31 set; its answer byte is never read).
// Packed images (fewer than 5 filters per group, 512 / 1,024 / 2,048 lines
// per slice) need offsets up to 2^11: the high 3 bits go to [26, 29), which
// a probe never reads either (only delta mod 512 matters).
constexpr uint32_t kEntryLineMask = 0xffu << 9;
constexpr uint32_t kEntryLineHiMask = 7u << 26;
constexpr uint32_t kProbePadEntry = 0x80000000u;
__device__ __forceinline__ uint32_t probe_entry(uint32_t h, uint32_t line_off) {
  return (h & ~(kEntryLineMask | kEntryLineHiMask | kProbePadEntry)) | ((line_off & 0xffu) << 9) |
         ((line_off >> 8) << 26);
}
__device__ __forceinline__ uint32_t probe_entry_off(uint32_t e) {
  return ((e >> 9) & 0xffu) | (((e >> 26) & 7u) << 8);
}
// One-pass multi-group entries: the probe's two 9-bit hash fields packed
// low -- h mod 512 in bits [0, 9), rotr(h, 17) mod 512 (hash bits [17, 26))
// in bits [9, 18) -- once per key, the line offset inside the slice (< 2^11)
// in bits [18, 29): one shift-or per group in the partition.  The slice pass
// reads only (x + q * (e >> 9)) mod 512, so the higher bits of either field
// never matter; padding is 0 (line 0, answers never read).
constexpr uint32_t kMGEntryOffShift = 18;
constexpr uint32_t kMGPadEntry = 0u;
__device__ __forceinline__ uint32_t mg_entry_hash(uint32_t h) { return (h & 0x1ffu) | ((h >> 8) & 0x3fe00u); }

// f(b) for every bucket b < n (n <= kMaxSlices + 1): one bucket per thread
// when the workgroup has enough threads.  A strided loop's per-lane trip
// count is a loop invariant the persistent partition spilled to scratch, and
// every scratch reload is an s_waitcnt vmcnt(0) that drained the key tiles
// in flight once per chunk.
template <int NT, typename F>
__device__ __forceinline__ void for_buckets(uint32_t n, F f) {
  if constexpr (NT > kMaxSlices) {
    if (threadIdx.x < n) f(threadIdx.x);
  } else {
    for (uint32_t b = threadIdx.x; b < n; b += NT) f(b);
  }
}

// Pass 1: hash each lookup once and bucket it by slice inside its chunk.
// entries[chunk region of probe_region(C) u32] = packed entries (probe_entry)
// grouped by slice, every bucket padded to a multiple of 4 entries with
// kProbePadEntry, so the slice pass moves whole 16-byte units; pos[i] = where
// key i went.  NT threads per chunk of C keys (C/NT keys per thread).
// NTS: non-temporal stores of the intermediates (default); plain stores
// leave them in the Infinity Cache for a round-sized batch to re-read.
// PERSIST: a grid smaller than the chunk count loops over the chunks with
// the next chunk's key tiles in flight; otherwise one workgroup per chunk
// (the default: no cross-chunk state to keep in registers).
template <int MODE, int NT, int C, int H = 1, bool NTS = true, bool PERSIST = true>
__global__ __launch_bounds__(NT, (NT <= 512 && H > 1) ? 4 : 1) void probe_partition_kernel(
    KeyDesc kd, uint32_t L, uint32_t magic, uint32_t R, uint32_t rmagic, uint32_t S, uint32_t nC,
    uint32_t* __restrict__ entries, uint16_t* __restrict__ pos, uint16_t* __restrict__ tab) {
  // H > 1: the chunk is hashed and bucketed in H units of CH keys (the tile
  // pipeline's unit stays CH), ranks keep counting across units, so every
  // bucket of the C-key chunk is one contiguous run: C-key chunks (longer
  // runs for the slice pass's gather) at the register cost of CH-key ones.
  // Entries of all but the last unit wait in LDS (`park`) until the chunk's
  // bucket offsets are known.
  constexpr int CH = C / H;
  constexpr int PER = CH / NT;
  constexpr uint32_t CR = probe_region(C);
  // the key tile doubles as the bucketed-entry staging area (CR u32)
  constexpr int KB = mode_kb<MODE>();
  constexpr int KPT = tile_kpt<KB>();
  using TL = K20Tile<NT, KPT, KB>;
  constexpr int TV = TL::kVec > static_cast<int>(CR / 4) ? TL::kVec : static_cast<int>(CR / 4);
  static_assert(PER % KPT == 0 && CR <= 65536 && C % H == 0, "chunk shape");
  __shared__ __attribute__((aligned(16))) uint4 tile[TV];
  __shared__ __attribute__((aligned(16))) uint16_t rk[C];  // rank in bucket, then position
  __shared__ uint8_t sb[C];                                // slice (S <= 256)
  __shared__ uint32_t park[H > 1 ? (H - 1) * CH : 1];      // entries of units 0..H-2
  __shared__ uint32_t hist[kMaxSlices + 1];
  __shared__ uint8_t npad[kMaxSlices + 1];
  __shared__ uint32_t wsum[NT / 64];
  const int tid = threadIdx.x;
  uint32_t* stage = reinterpret_cast<uint32_t*>(tile);
  auto chunk_keys = [&](uint32_t cc) {
    const uint64_t left = kd.n - static_cast<uint64_t>(cc) * C;
    return left < static_cast<uint64_t>(C) ? static_cast<uint32_t>(left) : static_cast<uint32_t>(C);
  };
  auto unit_keys = [&](uint32_t nk, int u) {  // keys of unit u of a chunk of nk keys
    const uint32_t b = static_cast<uint32_t>(u) * CH;
    return nk > b ? min(nk - b, static_cast<uint32_t>(CH)) : 0u;
  };
  // K20 / K28 (units of <= 8 keys per thread: more spills): the key tiles are
  // software-pipelined across units and chunks (hash_chunk_k20_pipe) -- one
  // resident workgroup per CU would otherwise leave its CU's HBM stream idle
  // during the bucket / scan / scatter / store phases.
  constexpr bool kPipe = (MODE == KM_K20 || MODE == KM_K28) && PER <= 8 && PER / KPT >= 2;
  uint4 pre[2][TL::kPer];
  if constexpr (kPipe) {
    if (blockIdx.x < nC) {
      const uint8_t* b0 = kd.bytes + static_cast<uint64_t>(blockIdx.x) * C * KB;
      const uint32_t n0 = unit_keys(chunk_keys(blockIdx.x), 0);
      k20_tile_fetch<NT, KPT, KB>(b0, n0 * KB, 0, pre[0]);
      if (n0 > static_cast<uint32_t>(TL::kKeys)) k20_tile_fetch<NT, KPT, KB>(b0, n0 * KB, 1, pre[1]);
    }
  }
  // grid-stride over chunks (a grid smaller than nC makes the pass persistent)
  for (uint32_t c = blockIdx.x; c < nC; c += PERSIST ? gridDim.x : nC) {
    const uint64_t first = static_cast<uint64_t>(c) * C;
    const uint32_t nk = chunk_keys(c);
    for_buckets<NT>(S + 1, [&](uint32_t b) { hist[b] = 0; });
    uint32_t h[PER];
#pragma unroll
    for (int u = 0; u < H; u++) {
      const uint32_t nku = unit_keys(nk, u);
      const uint64_t fu = first + static_cast<uint64_t>(u) * CH;
      if constexpr (kPipe) {
        const uint32_t cn = PERSIST ? c + gridDim.x : nC;  // the workgroup's next chunk, if any
        const uint64_t nf = u + 1 < H ? fu + CH : static_cast<uint64_t>(cn) * C;
        const uint32_t nn = u + 1 < H ? unit_keys(nk, u + 1) : (cn < nC ? unit_keys(chunk_keys(cn), 0) : 0u);
        hash_chunk_k20_pipe<NT, PER, KB>(kd, fu, nku, nf, nn, tile, h, pre);  // ends with a barrier
      } else {
        // K20 / K28 end with a barrier; KM_HASH / GENERIC load straight to
        // registers, so the bucket counters' zeroing above needs its own
        if constexpr (MODE == KM_HASH || MODE == KM_GENERIC) {
          if (u == 0) __syncthreads();
        }
        hash_chunk<MODE, NT, PER>(kd, fu, nku, tile, h);
      }
#pragma unroll
      for (int r = 0; r < PER; r++) {
        const uint32_t il = r * NT + tid;
        const uint32_t i = static_cast<uint32_t>(u) * CH + il;
        if (il < nku) {
          const uint32_t line = fastmod(h[r], L, magic);
          uint32_t off;  // slices of R lines (not a power of two when balanced over the CUs)
          const uint32_t sl = fastdivmod(line, R, rmagic, &off);
          sb[i] = static_cast<uint8_t>(sl);
          rk[i] = static_cast<uint16_t>(atomicAdd(&hist[sl], 1u));
          h[r] = probe_entry(h[r], off);
          if (u + 1 < H) park[i] = h[r];
        }
      }
    }
    __syncthreads();
    for_buckets<NT>(S, [&](uint32_t b) {  // pad every bucket to whole 16-byte units
      const uint32_t pad = (0u - hist[b]) & 3u;
      npad[b] = static_cast<uint8_t>(pad);
      hist[b] += pad;
    });
    __syncthreads();
    const uint32_t total = block_excl_scan_lds<NT>(hist, static_cast<int>(S + 1), wsum);
    for_buckets<NT>(S + 1, [&](uint32_t b) {  // one row per chunk
      tab[static_cast<uint64_t>(c) * (S + 1) + b] = static_cast<uint16_t>(hist[b]);
    });
    for_buckets<NT>(S, [&](uint32_t b) {
      const uint32_t end = hist[b + 1];
      const uint32_t np = npad[b];
      if (np > 0) stage[end - 1] = kProbePadEntry;
      if (np > 1) stage[end - 2] = kProbePadEntry;
      if (np > 2) stage[end - 3] = kProbePadEntry;
    });
    const uint32_t nkl = unit_keys(nk, H - 1);
#pragma unroll
    for (int r = 0; r < PER; r++) {  // the last unit, from registers
      const uint32_t il = r * NT + tid;
      const uint32_t i = static_cast<uint32_t>(H - 1) * CH + il;
      if (il < nkl) {
        const uint32_t p = hist[sb[i]] + rk[i];
        stage[p] = h[r];
        rk[i] = static_cast<uint16_t>(p);
      }
    }
    if constexpr (H > 1) {  // the parked units
      const uint32_t np = min(nk, static_cast<uint32_t>((H - 1) * CH));
      for (uint32_t i = tid; i < np; i += NT) {
        const uint32_t p = hist[sb[i]] + rk[i];
        stage[p] = park[i];
        rk[i] = static_cast<uint16_t>(p);
      }
    }
    __syncthreads();
    // The next unit's key tiles (issued before the bucketing) are waited for
    // HERE, while only loads are in flight: once the stores below are pending
    // every wait is a full vmcnt(0) that would also wait for their acks.
    if constexpr (kPipe) __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
    // coalesced 16-byte stores of the bucketed entries and of the positions
    store_chunk_u32<NT, NTS>(entries + static_cast<uint64_t>(c) * CR, stage, total);
    store_chunk_u16<NT, NTS>(pos + first, rk, nk);
    __syncthreads();  // LDS reused by the next chunk
  }
}

// A 16-byte load through a global-address-space pointer: an image pointer read
// from a descriptor in memory (the one-pass probe's MGroupDev) is generic, and
// generic (flat) loads of the slice made the compiler bounce them through
// scratch.
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
__device__ __forceinline__ uint4 ld_global16(const uint4* p) {
  const u32x4 x = *(g_u32x4*)(reinterpret_cast<uintptr_t>(p));
  return make_uint4(x.x, x.y, x.z, x.w);
}

// One probe of a packed image (LGW < 3): the W-bit field of position p in
// the line at LDS byte `base`, shifted down to bit 0 (higher bits are the
// next fields: the caller masks after the AND of the k probes).
template <int LGW>
__device__ __forceinline__ uint32_t packed_probe(const uint8_t* sl, uint32_t base, uint32_t x) {
  const uint32_t p = x & 511u;
  return static_cast<uint32_t>(sl[base + (p >> (3 - LGW))]) >> ((p << LGW) & 7u);
}
// The group's answer byte from a packed image's W-bit field: member m's bit
// goes to its slot bit (slotmap >> 4m) & 7.
template <int LGW>
__device__ __forceinline__ uint32_t packed_answer(uint32_t acc, uint32_t slotmap) {
  uint32_t a = 0;
#pragma unroll
  for (int m = 0; m < (1 << LGW); m++) a |= ((acc >> m) & 1u) << ((slotmap >> (4 * m)) & 7u);
  return a;
}

// Pass 2: one NT-thread workgroup per (slice of 2^LGR stacked lines, part of
// the chunks of C keys); the slice (R lines x 64 * 2^LGW B: 64 or 128 KiB)
// sits in LDS, waves walk the slice's segments of 64 chunks at a time.
// smask gets each key's answer byte at the key's bucketed position.
// LGW 3: byte-wide stacked image (up to 8 filters, one byte per bit position);
// LGW 0..2: packed image of a group of 1, 2 or 3-4 filters (a W-bit field per
// bit position: 8 / 4 / 2 times the lines per slice), whose member m answers
// in bit (slotmap >> 4m) & 7.
// plan (nullptr: every slice has `parts` parts): S+1 workgroup starts, slice
// s owning workgroups [plan[s], plan[s+1]) -- its parts, as many as its share
// of the entries asks for (version_plan_kernel); workgroups past plan[S] exit.
// MG (one-pass multi-group probe): the launch covers global slices
// [s0, s0 + S) of the groups mg[0, mg_n) (one image width LGW); each
// workgroup's slice names its group, whose image, L, R, k and slotmap replace
// the arguments; table rows hold `rowlen` offsets and chunk regions `cre_rt`
// entries (both known at run time only).
template <int LGR, int LGW, int K, int NT, int C, uint32_t CRE = probe_region(C), bool MG = false>
__global__ __launch_bounds__(NT, DLSM_PROBE_MINWAVES) void probe_slice_kernel(
    const uint8_t* __restrict__ stacked, uint32_t L, uint32_t Rs, uint32_t slotmap, int k, uint32_t S,
    uint32_t nC, const uint32_t* __restrict__ entries, const uint16_t* __restrict__ tab,
    uint8_t* __restrict__ smask, int parts, const uint32_t* __restrict__ plan = nullptr,
    const MGroupDev* __restrict__ mg = nullptr, int mg_n = 0, uint32_t s0 = 0, uint32_t rowlen = 0,
    uint32_t cre_rt = 0, uint32_t abytes = 0) {
  // LDS holds up to R = 2^LGR lines; a slice is Rs <= R lines (Rs < R when the
  // slices are balanced so that S x parts fills the CUs exactly)
  constexpr uint32_t R = 1u << LGR;
  constexpr uint32_t LB = 64u << LGW;  // bytes per line of the image
  static_assert(LGW == 3 || LGR + LGW == 11, "packed images use 128 KiB slices");
  // window units in flight per wave: one 128 KiB slice per CU (LGR 8) leaves
  // 4 waves per SIMD, so each carries two windows (measured best per shape)
  constexpr int U = LGR + LGW >= 11 ? kProbeWalkU8 : kProbeWalkU;
  constexpr int NW = NT / 64;
  __shared__ __attribute__((aligned(16))) uint8_t sl[R * LB];
  __shared__ uint32_t walk_scr[NW * kWalkScratch];
  const int tid = threadIdx.x;
  const int wv = wave_id();  // wave-uniform (SGPR): keeps the segment walk's control flow scalar
  const uint32_t wi = xcd_block(blockIdx.x, gridDim.x);
  uint32_t s, p;
  if (plan) {
    if (wi >= plan[S]) return;  // before any barrier: the whole workgroup leaves
    uint32_t lo = 0, hi = S - 1;  // the slice whose workgroup range holds wi
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (plan[mid] <= wi) lo = mid;
      else hi = mid - 1;
    }
    s = lo;
    p = wi - plan[s];
    parts = static_cast<int>(plan[s + 1] - plan[s]);
  } else {
    s = wi % S;
    p = wi / S;
  }
  uint32_t lo_line = s * Rs;
  uint32_t eoffu = 0, aoff = 0;  // MG: the group's entry sub-region (units), answer sub-area (bytes)
  if constexpr (MG) {
    s += s0;  // global slice
    int j = 0;
    for (int q = 1; q < mg_n; q++)
      if (mg[q].sbase <= s) j = q;  // groups in slice order
    stacked = mg[j].image;
    L = mg[j].L;
    Rs = mg[j].R;
    slotmap = mg[j].slotmap;
    k = mg[j].k;
    lo_line = (s - mg[j].sbase) * Rs;
    eoffu = mg[j].eoff / 4u;
    aoff = mg[j].aoff;
    s += static_cast<uint32_t>(j);  // the table column: every group has S_j + 1 columns
  } else {
    rowlen = S + 1;
  }
  const uint32_t nl = min(Rs, L - lo_line);
  // The slice into LDS: every 16-byte load in flight before the first LDS
  // store.  Loads AND stores are clamped (lanes past the slice rewrite its
  // last unit with the same bytes): a store under a branch let the compiler
  // sink each load into its branch, one HBM round trip per load.
  constexpr int V = R * (LB / 16) / NT;
  const uint4* src = reinterpret_cast<const uint4*>(stacked + static_cast<uint64_t>(lo_line) * LB);
  uint4* dst = reinterpret_cast<uint4*>(sl);
  const uint32_t nw = nl * (LB / 16);
  const uint32_t c_lo = static_cast<uint32_t>(static_cast<uint64_t>(p) * nC / parts);
  const uint32_t c_hi = static_cast<uint32_t>(static_cast<uint64_t>(p + 1) * nC / parts);
  if constexpr (MG) {
    if (c_lo >= c_hi) return;  // a plan sized for large batches: this part has no chunks (whole workgroup)
  }
  const uint16_t* tb = tab + s;  // chunk-major rows of `rowlen` u16
  constexpr uint32_t CRU_C = MG ? 0u : CRE / 4;  // chunk region stride in 16-byte units (0: run time)
  const uint32_t CRU = MG ? cre_rt / 4 : CRE / 4;
  const uint32_t cru_magic = MG ? fastmod_magic(CRU) : 0u;
  // Each lane takes one 16-byte unit (4 entries, bucket padding included) per
  // window, probes its 4 entries and writes their 4 answer bytes as one dword
  // (the answers mirror the entries' layout).
  const uint32_t gs = min(64u, max(1u, (c_hi - c_lo + NW - 1) / NW));  // chunks per wave group
  auto probe_set = [&](const uint4 (&hv)[U], const uint32_t (&idx)[U], const bool (&ok)[U], uint32_t g) {
        uint32_t* gmask = reinterpret_cast<uint32_t*>(smask) + static_cast<uint64_t>(g) * CRU;
        uint32_t ans[U];
        if constexpr (MG) {
          // One-pass probe: every unit's answers as W = 2^LGW bits per entry
          // (the image's field; a stacked byte is slot-mapped already) at the
          // group's answer sub-area: a 4W-bit value per unit, two units per
          // byte at W = 1 (bucket runs are padded to pairs of units, so lanes
          // 2m and 2m + 1 always hold the two units of one byte).
          constexpr int NE = 4 * U;
          constexpr uint32_t WM = LGW == 3 ? 0xffu : (1u << (1 << LGW)) - 1u;
          uint32_t xs[NE], ds[NE], bs[NE], acc[NE];
#pragma unroll
          for (int u = 0; u < U; u++) {
            const uint32_t e4[4] = {hv[u].x, hv[u].y, hv[u].z, hv[u].w};
#pragma unroll
            for (int j = 0; j < 4; j++) {
              xs[4 * u + j] = e4[j];                       // bits [0, 9): h mod 512
              ds[4 * u + j] = e4[j] >> 9;                  // bits [9, 18): rotr(h, 17) mod 512
              bs[4 * u + j] = (e4[j] >> kMGEntryOffShift) * LB;  // the line's image bytes
              acc[4 * u + j] = WM;
            }
          }
          auto probe1 = [&](int n) -> uint32_t {
            if constexpr (LGW == 3) return sl[bs[n] | (xs[n] & 511u)];
            else return packed_probe<LGW>(sl, bs[n], xs[n]);
          };
          if constexpr (K > 0) {
#pragma unroll
            for (int q = 0; q < K; q++)
#pragma unroll
              for (int n = 0; n < NE; n++) {
                acc[n] &= probe1(n);
                xs[n] += ds[n];
              }
          } else {
            for (int q = 0; q < k; q++)
#pragma unroll
              for (int n = 0; n < NE; n++) {
                acc[n] &= probe1(n);
                xs[n] += ds[n];
              }
          }
          const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
          for (int u = 0; u < U; u++) {
            uint32_t f = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) f |= (acc[4 * u + j] & WM) << (j << LGW);
            uint32_t uo;
            const uint32_t cq = fastdivmod(idx[u], CRU, cru_magic, &uo);
            const uint32_t ul = uo - eoffu;  // the unit inside the group's sub-region
            uint8_t* base = smask + static_cast<uint64_t>(g + cq) * abytes + aoff;
            // Stores are unconditional (see below): a lane past the window's
            // end holds a valid lane's unit and rewrites its answer.
            if constexpr (LGW == 3) {
              *reinterpret_cast<uint32_t*>(base + 4u * ul) = f;
            } else if constexpr (LGW == 2) {
              *reinterpret_cast<uint16_t*>(base + 2u * ul) = static_cast<uint16_t>(f);
            } else if constexpr (LGW == 1) {
              base[ul] = static_cast<uint8_t>(f);
            } else {
              // W = 1: the pair's byte from lanes 2m (low nibble) and 2m + 1; a
              // lane past the window's end rewrites lanes 0 / 1's byte (its
              // neighbour may hold another copy of lane 0's unit)
              const uint32_t nb = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(
                  0, static_cast<int>(f), 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]: lane ^ 1
              uint32_t pb = (lane & 1u) ? (nb | (f << 4)) : (f | (nb << 4));
              uint64_t ad = reinterpret_cast<uint64_t>(base + (ul >> 1));
              const uint32_t pb0 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(pb), 0));
              const uint32_t alo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(ad), 0));
              const uint32_t ahi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(ad >> 32), 0));
              if (!ok[u]) {
                pb = pb0;
                ad = (static_cast<uint64_t>(ahi) << 32) | alo;
              }
              *reinterpret_cast<uint8_t*>(ad) = static_cast<uint8_t>(pb);
            }
          }
          return;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
          const uint32_t e4[4] = {hv[u].x, hv[u].y, hv[u].z, hv[u].w};
          uint32_t a = 0;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            uint32_t x = e4[j];
            const uint32_t delta = x >> 17;            // low 9 bits of rotr(h, 17)
            if constexpr (LGW < 3) {
              const uint32_t base = probe_entry_off(x) * LB;
              uint32_t acc = ~0u;
              if constexpr (K > 0) {
#pragma unroll
                for (int q = 0; q < K; q++) {
                  acc &= packed_probe<LGW>(sl, base, x);
                  x += delta;
                }
              } else {
                for (int q = 0; q < k; q++) {
                  acc &= packed_probe<LGW>(sl, base, x);
                  x += delta;
                }
              }
              a |= packed_answer<LGW>(acc, slotmap) << (8 * j);
              continue;
            }
            const uint32_t base = x & ((R - 1u) << 9);  // line offset * 512 stacked bytes (probe_entry)
            uint32_t acc = 0xffu;
            if constexpr (K > 0) {
#pragma unroll
              for (int q = 0; q < K; q++) {
                acc &= sl[base | (x & 511u)];
                x += delta;
              }
            } else {
              for (int q = 0; q < k; q++) {
                acc &= sl[base | (x & 511u)];
                x += delta;
              }
            }
            a |= acc << (8 * j);
          }
          ans[u] = a;
        }
        // Stores are unconditional: a lane past the window's end holds the
        // index (and so the entries and the answer) of a valid lane of the same
        // set, so it rewrites that lane's dword with the same value.  A store
        // under a branch makes the compiler's wait for the next set's loads a
        // vmcnt(0) that also waits for these stores' acks (every path must
        // agree on the count).
#pragma unroll
        for (int u = 0; u < U; u++) gmask[idx[u]] = ans[u];
  };
  if constexpr (LGW == 3) {
    // byte-wide images: the slice load runs as the walk's prologue, after the
    // walk's first table-row loads are issued (one round trip fewer before
    // the first entries load: small batches)
    auto slice_to_lds = [&] {
      uint4 t[V];
#pragma unroll
      for (int v = 0; v < V; v++) t[v] = ld_global16(src + min(static_cast<uint32_t>(v * NT + tid), nw - 1u));
#pragma unroll
      for (int v = 0; v < V; v++) dst[min(static_cast<uint32_t>(v * NT + tid), nw - 1u)] = t[v];
      __syncthreads();
    };
    walk_segments<U, CRU_C, uint4, DLSM_PROBE_DEPTH, DLSM_PROBE_NTL != 0>(
        tb, rowlen, entries, c_lo + wv * gs, NW * gs, c_hi, gs, walk_scr + wv * kWalkScratch, probe_set,
        slice_to_lds, CRU);
  } else {
    // packed images: the same load in front of the walk (as the walk's
    // prologue the compiler kept t[] in scratch for these shapes)
    {
      uint4 t[V];
#pragma unroll
      for (int v = 0; v < V; v++) t[v] = ld_global16(src + min(static_cast<uint32_t>(v * NT + tid), nw - 1u));
#pragma unroll
      for (int v = 0; v < V; v++) dst[min(static_cast<uint32_t>(v * NT + tid), nw - 1u)] = t[v];
    }
    __syncthreads();
    walk_segments<U, CRU_C, uint4, DLSM_PROBE_DEPTH, DLSM_PROBE_NTL != 0>(
        tb, rowlen, entries, c_lo + wv * gs, NW * gs, c_hi, gs, walk_scr + wv * kWalkScratch, probe_set,
        NoPrologue{}, CRU);
  }
}

// Eight positions (16 bytes) of the unpermute: read once, non-temporal with
// DLSM_PROBE_NTL (see SegWalk).
__device__ __forceinline__ uint4 load_pos8(const uint16_t* p) {
#if DLSM_PROBE_NTL
  const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(x.x, x.y, x.z, x.w);
#else
  return *reinterpret_cast<const uint4*>(p);
#endif
}

// Pass 3: one workgroup per chunk: stage the chunk's bucketed answers in LDS
// (16-byte loads), gather them back to key order through pos (16-byte loads
// of 8 positions), store 8 answers per lane.
// VEC: 8-byte answer stores (mask 8-byte aligned); otherwise byte stores, for
// a caller's mask that starts anywhere (a sub-slice of a byte tensor).
template <int C, bool VEC>
__global__ __launch_bounds__(kBlock) void probe_unpermute_kernel(uint64_t n,
                                                                 const uint16_t* __restrict__ pos,
                                                                 const uint8_t* __restrict__ smask,
                                                                 uint8_t* __restrict__ mask) {
  constexpr uint32_t CR = probe_region(C);
  __shared__ __attribute__((aligned(16))) uint8_t sm[CR];
  const int tid = threadIdx.x;
  const uint64_t first = static_cast<uint64_t>(blockIdx.x) * C;
  const uint64_t left = n - first;
  const uint32_t nk = left < static_cast<uint64_t>(C) ? static_cast<uint32_t>(left) : C;
  // the chunk's answer region (bucket padding included; positions point into it)
  const uint32_t nvec = (min(CR, nk + 4u * kMaxSlices) + 15u) / 16u;
  const uint4* s4 = reinterpret_cast<const uint4*>(smask + static_cast<uint64_t>(blockIdx.x) * CR);
  // the chunk's positions are loaded first (they do not depend on the staged
  // answers): their round trip overlaps the answers' instead of following it
  constexpr int PI = C / (8 * kBlock);
  static_assert(C % (8 * kBlock) == 0, "whole position vectors per thread");
  uint4 pre[PI];
#pragma unroll
  for (int q = 0; q < PI; q++) {
    const uint32_t i0 = 8u * (static_cast<uint32_t>(q) * kBlock + tid);
    if (i0 + 8u <= nk) pre[q] = load_pos8(pos + first + i0);
  }
  for (uint32_t v = tid; v < nvec; v += kBlock) reinterpret_cast<uint4*>(sm)[v] = s4[v];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PI; q++) {
    const uint32_t i0 = 8u * (static_cast<uint32_t>(q) * kBlock + tid);
    if (i0 >= nk) break;
    if (i0 + 8u <= nk) {
      const uint4 pv = pre[q];
      const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 2; j++) {
        lo |= uint32_t(sm[pw[j] & 0xffffu]) << (16 * j);
        lo |= uint32_t(sm[pw[j] >> 16]) << (16 * j + 8);
        hi |= uint32_t(sm[pw[j + 2] & 0xffffu]) << (16 * j);
        hi |= uint32_t(sm[pw[j + 2] >> 16]) << (16 * j + 8);
      }
      if constexpr (VEC) {
        *reinterpret_cast<uint2*>(mask + first + i0) = make_uint2(lo, hi);
      } else {
#pragma unroll
        for (int b = 0; b < 4; b++) {
          mask[first + i0 + b] = static_cast<uint8_t>(lo >> (8 * b));
          mask[first + i0 + 4 + b] = static_cast<uint8_t>(hi >> (8 * b));
        }
      }
    } else {
      for (uint32_t i = i0; i < nk; i++) mask[first + i] = sm[pos[first + i]];
    }
  }
}

// ---------------------------------------------------------------------------
// One-pass probe of a multi-group filter set (round 6; bloom_internal.h,
// MGroupDev).  Version::Get walks filters of many line counts
// (db/version_set.cc:273-321): the set's groups each need their own bucketing,
// but the keys are read and hashed ONCE here, and one slice pass and one
// unpermute serve every group.
// ---------------------------------------------------------------------------

// A full chunk's keys hashed into h[] (key r*NT+t -> thread t, h[r]) with
// every load unconditional: tile rows past the tile are clamped to its last
// 16 bytes (re-read, never stored), hashes come in as plain dwords.  Loads
// under per-lane bounds checks made the compiler wait for each one right where
// it was issued (a register copy merging the in-bounds and tail paths), one
// HBM round trip per load.
template <int MODE, int NT, int PER>
__device__ __forceinline__ void hash_full_chunk(const KeyDesc& kd, uint64_t first, uint4* tile,
                                                uint32_t (&h)[PER]) {
  const int t = threadIdx.x;
  if constexpr (MODE == KM_K20 || MODE == KM_K28) {
    constexpr int KB = mode_kb<MODE>();
    constexpr int KPT = tile_kpt<KB>();
    using TL = K20Tile<NT, KPT, KB>;
    constexpr int NTILES = PER / KPT;
    const uint4* b4 = reinterpret_cast<const uint4*>(kd.bytes + first * KB);
    uint4 all[NTILES][TL::kPer];
#pragma unroll
    for (int q = 0; q < NTILES; q++)
#pragma unroll
      for (int v = 0; v < TL::kPer; v++) {
        const uint32_t u = min(static_cast<uint32_t>(v * NT + t), static_cast<uint32_t>(TL::kVec - 1));
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b4 + q * TL::kVec + u));
        all[q][v] = make_uint4(x.x, x.y, x.z, x.w);
      }
#pragma unroll
    for (int q = 0; q < NTILES; q++) {
#pragma unroll
      for (int v = 0; v < TL::kPer; v++) {
        const uint32_t u = v * NT + t;
        if (TL::kVec % NT == 0 || u < static_cast<uint32_t>(TL::kVec)) tile[u] = all[q][v];
      }
      __syncthreads();
      const uint32_t* w = reinterpret_cast<const uint32_t*>(tile);
#pragma unroll
      for (int j = 0; j < KPT; j++) h[q * KPT + j] = hash_k20_lds(w + (KB / 4) * (j * NT + t));
      __syncthreads();
    }
  } else if constexpr (MODE == KM_HASH) {
    const uint32_t* hp = reinterpret_cast<const uint32_t*>(kd.bytes) + first;
#pragma unroll
    for (int r = 0; r < PER; r++) h[r] = __builtin_nontemporal_load(hp + r * NT + t);
  } else {
#pragma unroll
    for (int r = 0; r < PER; r++) h[r] = key_hash<KM_GENERIC>(kd, first + r * NT + t);
  }
}

// Pass 1: one NT-thread workgroup per chunk of C keys.  The chunk is hashed
// once into registers, then bucketed by every group (the group's LDS
// histogram + ranks + scan, as probe_partition_kernel does for one group);
// group j's bucket runs (each padded to kMGPad entries) go to its own
// sub-region of the chunk's region, its S_j + 1 bucket starts to table
// columns tcol_j.. of the chunk's row, and pos[(chunk * G + j) * C + i] =
// key i's entry index inside the sub-region (bloom_internal.h, MGroupDev).
// The groups are bucketed P at a time (the phases of a set run once: ranks,
// scans, scatter, stores), every key's slice, rank and entry in registers (a
// full chunk's rank atomics issue back to back, one LDS wait).  Three
// barriers per set: after the ranks; after the scans -- wave p scans the
// set's group p, writes its table row and padding and zeroes its histogram of
// the next set (two sets of histograms alternate); after the scatter.  The
// slices are 2^lgR lines (a power of two in the one-pass layout), so a line's
// slice and offset are a shift and a mask.
#ifndef DLSM_MG_PWAVES
#define DLSM_MG_PWAVES 5  // partition: waves per SIMD the register budget must allow (A/B knob; 4: no spill, 1-2 % slower)
#endif
template <int MODE, int NT, int C, int P>
__global__ __launch_bounds__(NT, DLSM_MG_PWAVES) void probe_mpartition_kernel(KeyDesc kd, const MGroupDev* __restrict__ groups,
                                                              int G, uint32_t rowlen, uint32_t region,
                                                              uint32_t* __restrict__ entries,
                                                              uint16_t* __restrict__ pos,
                                                              uint16_t* __restrict__ tab) {
  constexpr int PER = C / NT;
  constexpr int KB = mode_kb<MODE>();
  constexpr int QB = (kMaxSlices + 1 + 63) / 64;  // buckets per lane of a scanning wave
  static_assert(PER % tile_kpt<KB>() == 0 && NT >= 64 * P, "chunk shape");
  // key tiles, then the set's staged entries (group p of a set at the sum of
  // the earlier groups' C + 8 S): dynamic LDS sized by the launcher for the
  // filter set's largest set (mg_stage_bytes), so the occupancy follows the
  // set's real padding, not the 256-slice worst case
  extern __shared__ __attribute__((aligned(16))) uint4 tile[];
  __shared__ __attribute__((aligned(16))) uint16_t rk[P][C];  // positions of the set's groups
  __shared__ uint32_t hist[2 * P][kMaxSlices + 1];           // counts, then starts: P per set, 2 sets
  const int tid = threadIdx.x;
  const uint32_t c = blockIdx.x;
  const uint64_t first = static_cast<uint64_t>(c) * C;
  const uint64_t left = kd.n - first;
  const uint32_t nk = left < static_cast<uint64_t>(C) ? static_cast<uint32_t>(left) : static_cast<uint32_t>(C);
  const bool full = nk == static_cast<uint32_t>(C);
  for (uint32_t b = tid; b < P * (kMaxSlices + 1u); b += NT) (&hist[0][0])[b] = 0;  // (more than NT buckets)
  uint32_t h[PER];
  if (full) hash_full_chunk<MODE, NT, PER>(kd, first, tile, h);
  else hash_chunk<MODE, NT, PER>(kd, first, nk, tile, h);
  __syncthreads();  // hist[0..P) zeroed (and, for hashes / generic keys, nothing else to wait for)
  uint32_t* stage = reinterpret_cast<uint32_t*>(tile);
  uint16_t* trow = tab + static_cast<uint64_t>(c) * rowlen;
  uint32_t* ereg = entries + static_cast<uint64_t>(c) * region;
  const uint32_t lane = tid & 63;
  const int wv = wave_id();
  // the part of every group's entry that does not depend on the group
  // (mg_entry): computed once per key
  uint32_t hk[PER];
#pragma unroll
  for (int r = 0; r < PER; r++) hk[r] = mg_entry_hash(h[r]);
  for (int j0 = 0, q = 0; j0 < G; j0 += P, q ^= 1) {
    const int np = min(P, G - j0);  // groups in this set (uniform)
    uint32_t pk[P][PER], e[P][PER];   // (rank << 8) | slice; the entry
#pragma unroll
    for (int pp = 0; pp < P; pp++) {
      if (pp >= np) break;
      const MGroupDev* gd = groups + j0 + pp;
      const uint32_t L = gd->L, magic = gd->magic, R = gd->R;
      const uint32_t lgR = static_cast<uint32_t>(__builtin_ctz(R));
      uint32_t* hc = hist[P * q + pp];
#pragma unroll
      for (int r = 0; r < PER; r++) {
        const uint32_t line = fastmod(h[r], L, magic);
        pk[pp][r] = line >> lgR;
        e[pp][r] = hk[r] | ((line & (R - 1u)) << kMGEntryOffShift);
      }
      if (full) {
#pragma unroll
        for (int r = 0; r < PER; r++) pk[pp][r] |= atomicAdd(&hc[pk[pp][r]], 1u) << 8;
      } else {
#pragma unroll
        for (int r = 0; r < PER; r++)
          if (static_cast<uint32_t>(r * NT + tid) < nk) pk[pp][r] |= atomicAdd(&hc[pk[pp][r]], 1u) << 8;
      }
    }
    __syncthreads();
    if (wv < np) {
      // wave p: exclusive scan of group j0+p's padded counts (QB buckets per
      // lane), its table row and padding; its histogram of the next set zeroed
      const int pp = wv;
      const MGroupDev* gd = groups + j0 + pp;
      const uint32_t S = gd->S, tcol = gd->tcol, eoff = gd->eoff;
      uint32_t* hc = hist[P * q + pp];
      uint32_t so = 0;  // the group's staging offset in the set
      for (int o = 0; o < pp; o++) so += mg_sub_entries(C, groups[j0 + o].S);
      uint32_t* st = stage + so;
      uint32_t cnt[QB], pc[QB], loc = 0;
#pragma unroll
      for (int k = 0; k < QB; k++) {
        const uint32_t b = QB * lane + k;
        cnt[k] = b < S ? hc[b] : 0u;
        pc[k] = (cnt[k] + (kMGPad - 1u)) & ~(kMGPad - 1u);
        loc += pc[k];
      }
      const uint32_t incl = wave_incl_scan(loc);
      uint32_t run = incl - loc;
#pragma unroll
      for (int k = 0; k < QB; k++) {
        const uint32_t b = QB * lane + k;
        if (b <= S) {
          hc[b] = run;
          trow[tcol + b] = static_cast<uint16_t>(eoff + run);
        }
        if (b < S)
          for (uint32_t p = run + cnt[k]; p < run + pc[k]; p++) st[p] = kMGPadEntry;
        run += pc[k];
      }
      if (j0 + P < G) {
#pragma unroll
        for (int k = 0; k < QB; k++)
          if (QB * lane + k <= static_cast<uint32_t>(kMaxSlices)) hist[P * (q ^ 1) + pp][QB * lane + k] = 0u;
      }
    }
    __syncthreads();
    uint32_t so = 0;  // staging offset of the set's group pp
#pragma unroll
    for (int pp = 0; pp < P; pp++) {
      if (pp >= np) break;
      const uint32_t* hc = hist[P * q + pp];
      uint32_t* st = stage + so;
      so += mg_sub_entries(C, groups[j0 + pp].S);
#pragma unroll
      for (int r = 0; r < PER; r++) {
        const uint32_t i = r * NT + tid;
        if (full || i < nk) {
          const uint32_t p = hc[pk[pp][r] & 0xffu] + (pk[pp][r] >> 8);
          st[p] = e[pp][r];
          rk[pp][i] = static_cast<uint16_t>(p);
        }
      }
    }
    __syncthreads();
#ifndef DLSM_MG_ABL
#define DLSM_MG_ABL 0  // ablation (timing only, wrong answers): 1 no entry stores, 2 no position stores
#endif
    so = 0;
#pragma unroll
    for (int pp = 0; pp < P; pp++) {
      if (pp >= np) break;
      const MGroupDev* gd = groups + j0 + pp;
      if constexpr (!(DLSM_MG_ABL & 1)) store_chunk_u32<NT, true>(ereg + gd->eoff, stage + so, hist[P * q + pp][gd->S]);
      if constexpr (!(DLSM_MG_ABL & 2)) store_chunk_u16<NT, true>(pos + (static_cast<uint64_t>(c) * G + j0 + pp) * C, rk[pp], nk);
      so += mg_sub_entries(C, gd->S);
    }
  }
}

// Pass 3: one workgroup per chunk: the chunk's answer area (every group's
// W_j-bit answers) staged in LDS, then per key (8 per lane per step) each
// group's answer field gathered through its position, mapped to its members'
// slot bits (a 16-entry table per packed group; a byte-wide stacked image's
// answer is the slot byte already) and OR-ed into the key's mask byte
// mask_byte_j.  Every mask byte is written whole: no memset, no
// read-modify-write.  MB: mask bytes per key (1 and 2 vectorized, 0 = any).
template <int C, int MB>
__global__ __launch_bounds__(kBlock) void probe_munpermute_kernel(uint64_t n, const MGroupDev* __restrict__ groups,
                                                                  int G, uint32_t abytes,
                                                                  const uint16_t* __restrict__ pos,
                                                                  const uint8_t* __restrict__ answers,
                                                                  uint8_t* __restrict__ mask, int mb) {
  extern __shared__ __attribute__((aligned(16))) uint8_t msm[];
  __shared__ uint8_t lut[kMGMaxGroups][16];  // packed group j: W-bit field -> slot bits
  const int tid = threadIdx.x;
  const uint32_t c = blockIdx.x;
  const uint64_t first = static_cast<uint64_t>(c) * C;
  const uint64_t left = n - first;
  const uint32_t nk = left < static_cast<uint64_t>(C) ? static_cast<uint32_t>(left) : static_cast<uint32_t>(C);
  const uint4* s4 = reinterpret_cast<const uint4*>(answers + static_cast<uint64_t>(c) * abytes);
  for (uint32_t v = tid; v < abytes / 16u; v += kBlock) reinterpret_cast<uint4*>(msm)[v] = s4[v];
  if (tid < kMGMaxGroups * 16) {
    const int j = tid >> 4;
    const uint32_t f = tid & 15u;
    uint32_t a = 0;
    if (j < G && groups[j].lgw < 3) {
      const uint32_t sm = groups[j].slotmap;
      for (int m = 0; m < (1 << groups[j].lgw); m++) a |= ((f >> m) & 1u) << ((sm >> (4 * m)) & 7u);
    }
    lut[j][f] = static_cast<uint8_t>(a);
  }
  __syncthreads();
  const uint16_t* pc = pos + static_cast<uint64_t>(c) * G * C;
  // the answer field of group j's entry pl, mapped to slot bits
  auto field = [&](int j, uint32_t lgw, uint32_t aoff, uint32_t pl) -> uint32_t {
    if (lgw == 3) return msm[aoff + pl];
    const uint32_t bit = pl << lgw;
    return lut[j][(msm[aoff + (bit >> 3)] >> (bit & 7u)) & ((1u << (1u << lgw)) - 1u)];
  };
  for (uint32_t i0 = 8u * tid; i0 < nk; i0 += 8u * kBlock) {
    if (i0 + 8u > nk) {  // the batch's ragged end: key by key
      for (uint32_t i = i0; i < nk; i++) {
        uint64_t a = 0;
        for (int j = 0; j < G; j++)
          a |= static_cast<uint64_t>(field(j, groups[j].lgw, groups[j].aoff, pc[static_cast<uint64_t>(j) * C + i]))
               << (8 * groups[j].mask_byte);
        for (int b = 0; b < mb; b++) mask[(first + i) * static_cast<uint64_t>(mb) + b] = static_cast<uint8_t>(a >> (8 * b));
      }
      break;
    }
    uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // key i0 + q's mask bytes
    for (int j = 0; j < G; j++) {
      const uint32_t sh = 8u * static_cast<uint32_t>(groups[j].mask_byte);
      const uint32_t lgw = static_cast<uint32_t>(groups[j].lgw), aoff = groups[j].aoff;
      const uint4 pv = load_pos8(pc + static_cast<uint64_t>(j) * C + i0);
      const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
      for (int q = 0; q < 4; q++) {
        acc[2 * q] |= static_cast<uint64_t>(field(j, lgw, aoff, pw[q] & 0xffffu)) << sh;
        acc[2 * q + 1] |= static_cast<uint64_t>(field(j, lgw, aoff, pw[q] >> 16)) << sh;
      }
    }
    if constexpr (MB == 1) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        lo |= static_cast<uint32_t>(acc[q] & 0xffu) << (8 * q);
        hi |= static_cast<uint32_t>(acc[q + 4] & 0xffu) << (8 * q);
      }
      *reinterpret_cast<uint2*>(mask + first + i0) = make_uint2(lo, hi);
    } else if constexpr (MB == 2) {
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; q++)
        w[q] = static_cast<uint32_t>(acc[2 * q] & 0xffffu) | (static_cast<uint32_t>(acc[2 * q + 1] & 0xffffu) << 16);
      *reinterpret_cast<uint4*>(mask + 2 * (first + i0)) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
#pragma unroll
      for (int q = 0; q < 8; q++)
        for (int b = 0; b < mb; b++)
          mask[(first + i0 + q) * static_cast<uint64_t>(mb) + b] = static_cast<uint8_t>(acc[q] >> (8 * b));
    }
  }
}

// ---------------------------------------------------------------------------
// MultiGet-style probe of a version: per lookup key,
// the files Version::ForEachOverlapping (db/version_set.cc:273-321) visits --
// level-0 files whose user-key range holds the key, newest first, then per
// level the file FindFile (:95-118) picks -- whose filter passes the key
// (Table::InternalGet, table/table.cc:350-358).  One thread per key; the key
// is hashed once (the reference re-hashes per file: same value).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int bytewise_cmp(const uint8_t* a, uint64_t an, const uint8_t* b, uint64_t bn) {
  // BytewiseComparator: memcmp over the shorter length, then the length
  const uint64_t n = an < bn ? an : bn;
  for (uint64_t j = 0; j < n; j++) {
    const int d = static_cast<int>(a[j]) - static_cast<int>(b[j]);
    if (d) return d;
  }
  return an < bn ? -1 : (an > bn ? 1 : 0);
}

// The first 16 bytes of a key, zero-padded, as two big-endian u64
// (VersionDev::pre_small / pre_large).  If two keys' prefixes differ, their
// order is the bytewise order of the keys: at the first differing byte either
// both keys have a byte there, or the shorter key has ended (a pad zero) and
// is a proper prefix of the longer one, which BytewiseComparator also orders
// first.  Equal prefixes need the full comparison.
template <int MODE>
__device__ __forceinline__ ulonglong2 key_prefix(const uint8_t* p, uint64_t len) {
  ulonglong2 r{0, 0};
  if (MODE == KM_K20 && len >= 16) {  // 4-byte aligned fixed 20-byte keys
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
    r.x = (static_cast<uint64_t>(__builtin_bswap32(w[0])) << 32) | __builtin_bswap32(w[1]);
    r.y = (static_cast<uint64_t>(__builtin_bswap32(w[2])) << 32) | __builtin_bswap32(w[3]);
    return r;
  }
  for (uint64_t i = 0; i < 16 && i < len; i++) {
    if (i < 8) r.x |= static_cast<uint64_t>(p[i]) << (56 - 8 * i);
    else r.y |= static_cast<uint64_t>(p[i]) << (56 - 8 * (i - 8));
  }
  return r;
}

__device__ __forceinline__ int cmp_prefix(const ulonglong2& a, const ulonglong2& b) {
  if (a.x != b.x) return a.x < b.x ? -1 : 1;
  if (a.y != b.y) return a.y < b.y ? -1 : 1;
  return 0;
}

// ROUTE: the sliced version probe's route pass -- a file of a sliced level
// (v.lvl_sliced[lv] = j >= 0) is not probed here; the lookup's global line in
// the level image goes to gl[j * n + i] instead (kVNoLine when the level has
// no candidate or the candidate has no filter), and its hash to hv[i].
template <int MODE, bool ROUTE = false>
__global__ __launch_bounds__(kBlock) void version_probe_kernel(VersionDev v, KeyDesc kd, uint64_t snapshot,
                                                               uint64_t* __restrict__ slot_mask,
                                                               uint32_t* __restrict__ level_file,
                                                               uint32_t* __restrict__ hv = nullptr,
                                                               uint32_t* __restrict__ gl = nullptr) {
  const uint64_t i = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x;
  if (i >= kd.n) return;
  uint64_t s, l;
  if (kd.offsets) {
    s = kd.offsets[i];
    l = kd.offsets[i + 1] - s;
  } else {
    s = i * kd.key_len;
    l = kd.key_len;
  }
  l = l > kd.suffix ? l - kd.suffix : 0;  // ExtractUserKey
  const uint8_t* uk = kd.bytes + s;
  const uint32_t h = key_hash<MODE>(kd, i);
  const ulonglong2 q = key_prefix<MODE>(uk, l);
  // BytewiseComparator order of the lookup user key against a file's
  // smallest / largest user key (prefixes first, the full keys on a tie)
  auto vs_small = [&](uint32_t f) {
    const int r = cmp_prefix(q, v.pre_small[f]);
    return r ? r : bytewise_cmp(uk, l, v.keyblob + v.files[f].smallest_off, v.files[f].smallest_len);
  };
  auto vs_large = [&](uint32_t f) {
    const int r = cmp_prefix(q, v.pre_large[f]);
    return r ? r : bytewise_cmp(uk, l, v.keyblob + v.files[f].largest_off, v.files[f].largest_len);
  };
  // LookupKey(user_key, snapshot): trailer PackSequenceAndType(snapshot, kValueTypeForSeek)
  const uint64_t tnum = (snapshot << 8) | 1u;
  uint64_t m = 0;
  for (uint32_t f = 0; f < v.n_l0; f++) {  // level 0: newest first
    if (vs_small(f) >= 0 && vs_large(f) <= 0) {
      const VFileDev& F = v.files[f];
      if (F.f.data == nullptr || full_may_match(h, F.f)) m |= 1ull << f;
    }
  }
  for (int lv = 1; lv < kNumLevels; lv++) {
    const uint32_t nf = v.lvl_count[lv];
    uint32_t pick = 0xffffffffu;
    uint32_t gline = kVNoLine;
    if (nf) {
      const uint32_t b = v.lvl_begin[lv];
      // FindFile: earliest file whose largest internal key >= the lookup key
      // (right starts at nf-1, so the last file is picked when none is >=)
      uint32_t left = 0, right = nf - 1;
      while (left < right) {
        const uint32_t mid = (left + right) / 2;
        int r = -vs_large(b + mid);  // largest vs lookup
        if (r == 0) {
          const uint64_t tr = v.files[b + mid].largest_trailer;
          r = tr > tnum ? -1 : (tr < tnum ? 1 : 0);
        }
        if (r < 0) left = mid + 1;
        else right = mid;
      }
      if (vs_small(b + right) >= 0) {
        pick = right;
        const VFileDev& F = v.files[b + right];
        if (ROUTE && v.lvl_sliced[lv] >= 0 && F.f.data != nullptr)
          gline = F.line0 + fastmod(h, F.f.L, F.f.magic);
        else if (F.f.data == nullptr || full_may_match(h, F.f))
          m |= 1ull << (v.n_l0 + lv - 1);
      }
    }
    if (level_file) level_file[i * (kNumLevels - 1) + (lv - 1)] = pick;
    if (ROUTE && v.lvl_sliced[lv] >= 0) gl[static_cast<uint64_t>(v.lvl_sliced[lv]) * kd.n + i] = gline;
  }
  slot_mask[i] = m;
  if (ROUTE) hv[i] = h;
}

// The version probe with the version's interval index in LDS (a persistent
// grid: each workgroup copies it once).  A lookup finds its open interval
// with one branchless binary search over the bound prefixes (VersionDev::bnd)
// and reads which level-0 files hold it and each level's FindFile pick from
// the interval's record: the reference's per-level searches and level-0
// range checks (Version::ForEachOverlapping, db/version_set.cc:273-321) are
// resolved once per version, at dlsm_version_create, instead of per lookup.
// A lookup whose prefix equals a bound prefix (it equals a file's smallest /
// largest user key, or shares 16 bytes with one) takes the full comparison
// path, including FindFile's internal-key tie-break on the snapshot.
// ROUTE as in version_probe_kernel.
//
// Direct probes (level-0 files, and levels probed directly) do not run where
// a lane finds them: a scattered load costs the vector memory pipeline about
// one cycle per cache line it touches whatever the exec mask, and each probe
// site of a lane-per-lookup loop is a chain of up to k such loads with most
// lanes idle.  Instead every lane appends its probe tasks (file, slot, lane)
// to a wave-private queue in LDS, and the wave answers them 64 at a time:
// the task lines are fetched four lanes per line, each lane one 16-byte
// quarter -- so one load instruction covers 16 whole lines -- and staged in
// LDS, then every lane tests its own task's k bits there and ORs the answer
// into the owning lane's slot mask (LDS).
struct VMeta {  // 32 B per file
  const uint8_t* data;
  uint32_t L, magic, line0;
  int32_t k, lg;
  uint32_t pad;
};
constexpr int kVRouteNT = 1024;           // 16 waves, one workgroup per CU (the LDS below)
constexpr int kVRouteWaves = kVRouteNT / 64;
constexpr int kVRound = 128;              // tasks per round: two 64-line halves' loads in flight
constexpr int kVQueue = kVRound + 64;     // queued probe tasks per wave (one enqueue adds <= 64)
// per wave: staged task lines (one half) | queued tasks' line addresses |
// queued task words | owning lanes' hashes | their answer masks
constexpr size_t kVWaveLds = 64 * 64 + kVQueue * 8 + kVQueue * 4 + 64 * 4 + 64 * 8;
constexpr size_t kVLdsMax = 160u * 1024u;  // the CU's LDS

constexpr uint32_t kVSparse = 8;  // bounds per global window of the sparse bound index (128 B)

size_t version_lds_bytes(uint32_t n_bnd, uint32_t nf, int gt) {  // gt: version_lds_kernel's GT
  size_t tables = 0;
  if (gt <= 1) tables += static_cast<size_t>(n_bnd) * 16u;
  if (gt <= 2) tables += static_cast<size_t>(nf) * sizeof(VMeta);
  if (gt == 0) tables += (static_cast<size_t>(n_bnd) + 1u) * sizeof(VIntervalDev);
  if (gt == 2 || gt == 3) tables += static_cast<size_t>((n_bnd + kVSparse - 1) / kVSparse) * 16u;
  return ((tables + 63u) & ~static_cast<size_t>(63u)) + kVRouteWaves * kVWaveLds;
}

// FullFilterBlockReader::KeyMayMatch (full_filter_block.cc:269-284) for one
// lane (files whose "lines" are not 64 bytes: the reader's log2 0 branch).
__device__ __forceinline__ uint32_t full_may_match_all(uint32_t h, const VMeta& f) {
  FilterDev g{f.data, f.L, f.magic, f.k, f.lg};
  return full_may_match(h, g);
}

// GT: how much of the version's tables the LDS holds, in the order they
// matter (measured: profiles/r05_t, r05_u_version_table_tiers.txt): the file
// metadata (read per probe task, inside every round's chain), the bound
// prefixes (the search's chain of dependent reads), the interval records
// (one read per lookup).  0: all three (up to ~440 files beside the wave
// queues); 1: the metadata and the prefixes (~770 files); 2: the metadata
// and every kVSparse-th prefix (~1,350 files); 3: every kVSparse-th prefix
// (~12,000 files); 4: none.  What the LDS does not hold is read from
// global memory, where it stays in L2; with the sparse prefixes the search
// ends in one window of kVSparse global prefixes read together (one L2
// round trip instead of a chain of log2(n_bnd)).  The probes go through the
// wave queues either way.
template <int MODE, bool ROUTE, int K, int GT>
__global__ __launch_bounds__(kVRouteNT) void version_lds_kernel(VersionDev v, KeyDesc kd, uint64_t snapshot,
                                                                uint64_t* __restrict__ slot_mask,
                                                                uint32_t* __restrict__ level_file,
                                                                uint32_t* __restrict__ hv, uint32_t* __restrict__ gl,
                                                                uint32_t nf) {
  extern __shared__ uint4 vdyn[];
  const uint32_t nb = v.n_bnd;
  constexpr bool kMeta = GT <= 2, kBnd = GT <= 1, kIvl = GT == 0, kSp = GT == 2 || GT == 3;
  const uint32_t nsp = kSp ? (nb + kVSparse - 1) / kVSparse : 0u;  // sparse prefixes
  ulonglong2* lbnd = reinterpret_cast<ulonglong2*>(vdyn);
  ulonglong2* lsp = lbnd + (kBnd ? nb : 0u);
  VMeta* lmeta = reinterpret_cast<VMeta*>(lsp + nsp);
  VIntervalDev* livl = reinterpret_cast<VIntervalDev*>(lmeta + (kMeta ? nf : 0u));
  // the wave areas start 64-byte aligned (ds_write_b128 staging; the 24-byte
  // interval records leave the tables' end 8-byte aligned only)
  uint8_t* wbase = reinterpret_cast<uint8_t*>(vdyn) +
                   ((reinterpret_cast<uint8_t*>(livl + (kIvl ? nb + 1u : 0u)) - reinterpret_cast<uint8_t*>(vdyn) + 63u) &
                    ~static_cast<size_t>(63u));
  const ulonglong2* bnd;
  const VIntervalDev* ivl;
  if constexpr (kBnd) bnd = lbnd;
  else bnd = v.bnd;
  if constexpr (kIvl) ivl = livl;
  else ivl = v.ivl;
  auto meta_at = [&](uint32_t f) -> VMeta {
    if constexpr (kMeta) {
      return lmeta[f];
    } else {
      const VFileDev& F = v.files[f];
      return VMeta{F.f.data, F.f.L, F.f.magic, F.line0, F.f.k, F.f.lg, 0u};
    }
  };
  const uint32_t lane = threadIdx.x & 63u;
  const int wv = wave_id();
  uint8_t* wl = wbase + static_cast<size_t>(wv) * kVWaveLds;
  typedef __attribute__((address_space(3))) uint32_t lds32;
  typedef __attribute__((address_space(3))) unsigned long long lds64;
  lds32* st = (lds32*)reinterpret_cast<uint32_t*>(wl);                                // 64 lines of 64 B
  lds64* ad = (lds64*)reinterpret_cast<unsigned long long*>(wl + 4096);              // kVQueue line addresses
  lds32* tq = (lds32*)reinterpret_cast<uint32_t*>(wl + 4096 + kVQueue * 8);
  lds32* hb = (lds32*)reinterpret_cast<uint32_t*>(wl + 4096 + kVQueue * 8 + kVQueue * 4);
  lds64* mb = (lds64*)reinterpret_cast<unsigned long long*>(wl + 4096 + kVQueue * 8 + kVQueue * 4 + 64 * 4);
  if constexpr (kBnd)
    for (uint32_t f = threadIdx.x; f < nb; f += kVRouteNT) lbnd[f] = v.bnd[f];
  if constexpr (kSp)  // window w's last prefix (the table's last for a short last window)
    for (uint32_t w = threadIdx.x; w < nsp; w += kVRouteNT) lsp[w] = v.bnd[min(w * kVSparse + kVSparse - 1u, nb - 1u)];
  if constexpr (kMeta)
    for (uint32_t f = threadIdx.x; f < nf; f += kVRouteNT) {
      const VFileDev& F = v.files[f];
      lmeta[f] = VMeta{F.f.data, F.f.L, F.f.magic, F.line0, F.f.k, F.f.lg, 0u};
    }
  if constexpr (kIvl)
    for (uint32_t f = threadIdx.x; f <= nb; f += kVRouteNT) livl[f] = v.ivl[f];
  mb[lane] = 0ull;
  __syncthreads();
  const uint64_t tnum = (snapshot << 8) | 1u;  // LookupKey(user_key, snapshot): kValueTypeForSeek
  // One round: tasks tq[0, n), n <= kVRound, wave-uniform, their line
  // addresses in ad[0, n) (written by the lane that queued each task).  Every
  // line is fetched four lanes per line (lane & 3 = its 16-byte quarter),
  // both halves' loads in flight at once; each half is staged in LDS in turn
  // and lane t tests task t + 64 hf's k bits there.
  auto round = [&](uint32_t n) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    uint32_t task[2], h[2];
#pragma unroll
    for (int hf = 0; hf < 2; hf++) {
      const uint32_t t = lane + 64u * hf;
      task[hf] = t < n ? tq[t] : ~0u;
    }
    const uint32_t qq = lane & 3u;
    // global (not flat) 16-byte loads, 16-byte LDS stores
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(1))) const v4u gv4u;
    typedef __attribute__((address_space(3))) v4u lv4u;
    v4u qv[8];
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const uint32_t t = 16u * r + (lane >> 2);
      qv[r] = v4u{0u, 0u, 0u, 0u};
      // default cache policy: the level-0 / level-1 lines are L2 hits (with
      // the non-temporal hint they miss: 2.1 x slower, r05_p_version_line_nt_ab.txt)
      if (t < n) qv[r] = *(gv4u*)(ad[t] + 16u * qq);
    }
    // the owning lanes' hashes, read while the lines are in flight
#pragma unroll
    for (int hf = 0; hf < 2; hf++) h[hf] = task[hf] != ~0u ? hb[task[hf] >> 26] : 0u;
#pragma unroll
    for (int hf = 0; hf < 2; hf++) {
      if (64u * hf >= n) break;  // wave-uniform
#pragma unroll
      for (int r = 4 * hf; r < 4 * hf + 4; r++) {
        const uint32_t t = 16u * r + (lane >> 2);
        if (t < n) *(lv4u*)(st + (t - 64u * hf) * 16u + qq * 4u) = qv[r];
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      if (task[hf] != ~0u) {
        // HashMayMatchPrepared, bloom_impl.h:466-479, on the staged line
        const lds32* line = st + lane * 16u;
        uint32_t hh = h[hf];
        const uint32_t delta = bloom_delta(hh);
        uint32_t bad = 0u;
        if constexpr (K > 0) {
          // all K reads issued before the first use: one LDS round trip, not K
          uint32_t w[K], sh[K];
#pragma unroll
          for (int q = 0; q < K; q++, hh += delta) {
            sh[q] = hh;
            w[q] = line[(hh >> 5) & 15u];
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int q = 0; q < K; q++) bad |= ~w[q] >> (sh[q] & 31u);
        } else {
          const int kk = meta_at(task[hf] & 0xffffu).k;
          for (int q = 0; q < kk; q++, hh += delta) bad |= ~line[(hh & 511u) >> 5] >> (hh & 31u);
        }
        if (!(bad & 1u)) atomicOr((unsigned long long*)&mb[task[hf] >> 26], 1ull << ((task[hf] >> 16) & 63u));
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
  };
  const uint64_t wstride = static_cast<uint64_t>(gridDim.x) * kVRouteWaves * 64u;
  const uint64_t base0 = (static_cast<uint64_t>(blockIdx.x) * kVRouteWaves + wv) * 64u;
  // K20: the next iteration's key words are loaded at the top of this one
  // and digested (hash, prefix) at its bottom, so the HBM round trip of the
  // key stream overlaps the searches and probe rounds, and what crosses the
  // loop's back edge is the digest, not the loaded registers (a loaded
  // register carried across it makes the compiler copy it -- and wait for
  // the load -- right where it is issued)
  uint32_t xn[5] = {0u, 0u, 0u, 0u, 0u};
  uint32_t hn = 0u;
  ulonglong2 qn = make_ulonglong2(0ull, 0ull);
  auto key_words = [&](uint64_t b, uint32_t (&x)[5]) {
    const uint64_t ii = min(b + lane, kd.n - 1);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(kd.bytes + ii * 20u);
#pragma unroll
    for (int j = 0; j < 5; j++) x[j] = __builtin_nontemporal_load(w + j);
  };
  auto digest = [&](const uint32_t (&x)[5]) {  // one read of the key's five words: hash and prefix
    hn = hash_init(20, kBloomSeed);
#pragma unroll
    for (int j = 0; j < 5; j++) hn = hash_word(hn, x[j]);
    qn.x = (static_cast<uint64_t>(__builtin_bswap32(x[0])) << 32) | __builtin_bswap32(x[1]);
    qn.y = (static_cast<uint64_t>(__builtin_bswap32(x[2])) << 32) | __builtin_bswap32(x[3]);
  };
  if constexpr (MODE == KM_K20) {
    if (base0 < kd.n) {
      key_words(base0, xn);
      digest(xn);
    }
  }
  for (uint64_t base = base0; base < kd.n; base += wstride) {
    const uint64_t i = base + lane;
    const bool live = i < kd.n;
    const uint64_t ii = live ? i : kd.n - 1;  // a dead lane reads a valid key and stores nothing
    uint64_t s, l;
    if (kd.offsets) {
      s = kd.offsets[ii];
      l = kd.offsets[ii + 1] - s;
    } else {
      s = ii * kd.key_len;
      l = kd.key_len;
    }
    l = l > kd.suffix ? l - kd.suffix : 0;  // ExtractUserKey
    const uint8_t* uk = kd.bytes + s;
    uint32_t h;
    ulonglong2 q;
    if constexpr (MODE == KM_K20) {
      h = hn;
      q = qn;
      if (base + wstride < kd.n) key_words(base + wstride, xn);
    } else {
      h = key_hash<MODE>(kd, ii);
      q = key_prefix<MODE>(uk, l);
    }
    hb[lane] = h;
    // the open interval: j = bounds below the lookup's prefix (a lower bound
    // whose halving steps depend on nb only: the same for every lane).  A
    // 4-ary form (three pivots per step read together, half the LDS round
    // trips) measured 1-2 % slower: its extra compares cost more VALU than
    // the round trips it saves (profiles/r05_version_probe_ab.txt).
    auto below = [&](const ulonglong2& p) -> uint32_t {
      return (p.x < q.x || (p.x == q.x && p.y < q.y)) ? 1u : 0u;
    };
    uint32_t j = 0;
    if constexpr (kSp) {
      // the sparse prefixes in LDS pick the window (windows whose last prefix
      // is below q), then the window's kVSparse prefixes, read together from
      // global memory, are counted: window c's last prefix is not below q, so
      // j lies inside it (a clamped read repeats the table's last prefix,
      // which is not below q either)
      uint32_t c = 0;
      if (nsp) {
        uint32_t len = nsp;
        while (len > 1) {
          const uint32_t half = len >> 1;
          if (below(lsp[c + half - 1])) c += half;
          len -= half;
        }
        c += below(lsp[c]);
      }
      if (c >= nsp) {
        j = nb;
      } else {
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        typedef __attribute__((address_space(1))) const u64x2 gu2;  // global, not flat, loads
        const gu2* gb = (const gu2*)v.bnd;
        u64x2 win[kVSparse];
#pragma unroll
        for (uint32_t k = 0; k < kVSparse; k++) win[k] = gb[min(c * kVSparse + k, nb - 1u)];
        j = c * kVSparse;
#pragma unroll
        for (uint32_t k = 0; k < kVSparse; k++) j += below(make_ulonglong2(win[k].x, win[k].y));
      }
    } else if (nb) {
      uint32_t len = nb;
      while (len > 1) {
        const uint32_t half = len >> 1;
        if (below(bnd[j + half - 1])) j += half;
        len -= half;
      }
      j += below(bnd[j]);
    }
    // the interval's record and the bound at j, read together (ivl has nb + 1)
    const ulonglong2 bj = bnd[min(j, nb ? nb - 1 : 0u)];
    const VIntervalDev R = ivl[j];
    const bool exact = j < nb && bj.x == q.x && bj.y == q.y;
    uint64_t l0m;
    uint32_t pick[kNumLevels - 1];
    if (!exact) {
      l0m = R.l0mask;
#pragma unroll
      for (int lv = 0; lv < kNumLevels - 1; lv++) pick[lv] = R.pick[lv] == 0xffffu ? 0xffffffffu : R.pick[lv];
    } else {
      // the full comparisons (version_probe_kernel's), tables in global memory
      auto vs_small = [&](uint32_t f) {
        const int r = cmp_prefix(q, v.pre_small[f]);
        return r ? r : bytewise_cmp(uk, l, v.keyblob + v.files[f].smallest_off, v.files[f].smallest_len);
      };
      auto vs_large = [&](uint32_t f) {
        const int r = cmp_prefix(q, v.pre_large[f]);
        return r ? r : bytewise_cmp(uk, l, v.keyblob + v.files[f].largest_off, v.files[f].largest_len);
      };
      l0m = 0;
      for (uint32_t f = 0; f < v.n_l0; f++)
        if (vs_small(f) >= 0 && vs_large(f) <= 0) l0m |= 1ull << f;
      for (int lv = 1; lv < kNumLevels; lv++) {
        pick[lv - 1] = 0xffffffffu;
        const uint32_t nf_l = v.lvl_count[lv];
        if (!nf_l) continue;
        const uint32_t b = v.lvl_begin[lv];
        uint32_t left = 0, right = nf_l - 1;
        while (left < right) {
          const uint32_t mid = (left + right) / 2;
          int r = -vs_large(b + mid);
          if (r == 0) {
            const uint64_t tr = v.files[b + mid].largest_trailer;
            r = tr > tnum ? -1 : (tr < tnum ? 1 : 0);
          }
          if (r < 0) left = mid + 1;
          else right = mid;
        }
        if (vs_small(b + right) >= 0) pick[lv - 1] = b + right;
      }
    }
    if (!live) l0m = 0;
    uint64_t m = 0;
    uint32_t queued = 0;  // wave-uniform
    // a direct probe of file f for slot `slot` (this lane, if `want`): queued;
    // a full queue answers a round of 64
    // the queueing lane writes its task's line address too (it holds the
    // file's metadata and its hash): a round reads the addresses in one LDS
    // round trip instead of three
    auto enqueue = [&](bool want, uint32_t f, uint32_t slot, const VMeta& F) {
      const uint64_t b = __ballot(want);
      if (!b) return;
      if (want) {
        const uint32_t below = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(b >> 32),
                                                         __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(b), 0u));
        tq[queued + below] = (lane << 26) | (slot << 16) | f;
        ad[queued + below] = reinterpret_cast<unsigned long long>(F.data + (fastmod(h, F.L, F.magic) << 6));
      }
      queued += static_cast<uint32_t>(__builtin_popcountll(b));
      if (queued >= static_cast<uint32_t>(kVRound)) {
        round(kVRound);
        const uint32_t rest = queued - kVRound;  // move the overflow (< 64) to the front
        const uint32_t t = lane < rest ? tq[kVRound + lane] : 0u;
        const unsigned long long a = lane < rest ? ad[kVRound + lane] : 0ull;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (lane < rest) {
          tq[lane] = t;
          ad[lane] = a;
        }
        queued = rest;
      }
    };
    const uint64_t anyl0 = uniform64(__ballot(l0m != 0));
    for (uint32_t f = 0; anyl0 && f < v.n_l0; f++) {  // level 0: newest first
      const bool in = (l0m >> f) & 1u;
      const VMeta F = meta_at(f);
      if (in && F.data == nullptr) m |= 1ull << f;
      if (in && F.data != nullptr && F.lg != 6 && full_may_match_all(h, F)) m |= 1ull << f;  // rare: 1-byte lines
      enqueue(in && F.data != nullptr && F.lg == 6, f, f, F);
    }
    // metadata in global memory: every level's pick read up front, the loads
    // in flight together (inside the loop each would wait behind the
    // previous level's enqueue)
    VMeta FP[kNumLevels - 1];
    if constexpr (!kMeta) {
#pragma unroll
      for (int lv = 1; lv < kNumLevels; lv++) {
        const uint32_t pf = live && v.lvl_count[lv] ? pick[lv - 1] : 0xffffffffu;
        FP[lv - 1] = pf != 0xffffffffu ? meta_at(pf) : VMeta{};
      }
    }
    for (int lv = 1; lv < kNumLevels; lv++) {
      const uint32_t slot = v.n_l0 + lv - 1;
      const uint32_t pf = live && v.lvl_count[lv] ? pick[lv - 1] : 0xffffffffu;
      uint32_t gline = kVNoLine;
      bool task = false;
      VMeta F{};
      if (pf != 0xffffffffu) {
        if constexpr (kMeta) F = meta_at(pf);
        else F = FP[lv - 1];
        if (ROUTE && v.lvl_sliced[lv] >= 0 && F.data != nullptr) {
          gline = F.line0 + fastmod(h, F.L, F.magic);
        } else if (F.data == nullptr) {
          m |= 1ull << slot;
        } else if (F.lg != 6) {
          if (full_may_match_all(h, F)) m |= 1ull << slot;
        } else {
          task = true;
        }
      }
      enqueue(task, pf, slot, F);
      if (live && level_file)
        level_file[i * (kNumLevels - 1) + (lv - 1)] = pf == 0xffffffffu ? pf : pf - v.lvl_begin[lv];
      if (ROUTE && live && v.lvl_sliced[lv] >= 0) gl[static_cast<uint64_t>(v.lvl_sliced[lv]) * kd.n + i] = gline;
    }
    if (queued) round(queued);
    m |= mb[lane];
    mb[lane] = 0ull;
    if (live) {
      slot_mask[i] = m;
      if (ROUTE) hv[i] = h;
    }
    if constexpr (MODE == KM_K20) {
      if (base + wstride < kd.n) digest(xn);
    }
  }
}

// Sliced version probe, partition pass (one NT-thread workgroup per chunk of
// kVChunk lookups): each lookup whose global line g lies in this pass's
// slices [g0, g0 + S << kVSliceLg) gets the entry probe_entry(h, line offset
// in its slice), bucketed by slice inside the chunk's region, every bucket
// padded to whole 16-byte units (the slice pass's unit); pos[i] = the entry's
// position in the region, kVNoPos for a lookup without a probe in this pass.
template <int NT>
__global__ __launch_bounds__(NT) void version_partition_kernel(const uint32_t* __restrict__ hv,
                                                               const uint32_t* __restrict__ gl, uint64_t n,
                                                               uint32_t g0, uint32_t S,
                                                               uint32_t* __restrict__ entries,
                                                               uint16_t* __restrict__ pos,
                                                               uint16_t* __restrict__ tab,
                                                               uint32_t* __restrict__ gcnt) {
  constexpr int C = kVChunk;
  constexpr int PER = C / NT;
  __shared__ __attribute__((aligned(16))) uint32_t stage[kVRegion];
  __shared__ uint32_t hist[kVMaxSlices + 1];
  __shared__ uint8_t npad[kVMaxSlices];
  __shared__ uint32_t wsum[NT / 64];
  const int tid = threadIdx.x;
  const uint32_t c = blockIdx.x;
  const uint64_t first = static_cast<uint64_t>(c) * C;
  const uint32_t nk = static_cast<uint32_t>(min(static_cast<uint64_t>(C), n - first));
  for (uint32_t b = tid; b <= S; b += NT) hist[b] = 0;
  uint32_t e[PER], sr[PER];  // entry; slice << 16 | rank (~0: no probe)
#pragma unroll
  for (int r = 0; r < PER; r++) {  // coalesced dword loads, all in flight before the barrier
    const uint32_t i = r * NT + tid;
    e[r] = i < nk ? __builtin_nontemporal_load(hv + first + i) : 0u;
    sr[r] = i < nk ? __builtin_nontemporal_load(gl + first + i) : kVNoLine;
  }
  __syncthreads();
  const uint32_t span = S << kVSliceLg;
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const uint32_t d = sr[r] - g0;
    if (sr[r] != kVNoLine && d < span) {
      const uint32_t sl = d >> kVSliceLg;
      sr[r] = (sl << 16) | atomicAdd(&hist[sl], 1u);
      e[r] = probe_entry(e[r], d & ((1u << kVSliceLg) - 1u));
    } else {
      sr[r] = ~0u;
    }
  }
  __syncthreads();
  for (uint32_t b = tid; b < S; b += NT) {  // whole 16-byte units
    const uint32_t pad = (0u - hist[b]) & 3u;
    npad[b] = static_cast<uint8_t>(pad);
    hist[b] += pad;
    if (hist[b]) atomicAdd(&gcnt[b], hist[b] >> 2);  // the slice's units, for the slice pass's plan
  }
  __syncthreads();
  const uint32_t total = block_excl_scan_lds<NT>(hist, static_cast<int>(S + 1), wsum);
  for (uint32_t b = tid; b <= S; b += NT) tab[static_cast<uint64_t>(c) * (S + 1) + b] = static_cast<uint16_t>(hist[b]);
  // padding entries (bit 31 set: never answered) at the end of every bucket;
  // the bucket's own entries fill the rest below
  for (uint32_t b = tid; b < S; b += NT) {
    const uint32_t end = hist[b + 1];
    for (uint32_t q = end - npad[b]; q < end; q++) stage[q] = kProbePadEntry;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const uint32_t i = r * NT + tid;
    if (i >= nk) continue;
    uint16_t p = kVNoPos;
    if (sr[r] != ~0u) {
      const uint32_t q = hist[sr[r] >> 16] + (sr[r] & 0xffffu);
      stage[q] = e[r];
      p = static_cast<uint16_t>(q);
    }
    pos[first + i] = p;
  }
  __syncthreads();
  store_chunk_u32<NT, true>(entries + static_cast<uint64_t>(c) * kVRegion, stage, total);
}

// Sliced version probe, slice plan (one workgroup): every slice gets
// max(1, ceil(units / target)) workgroup parts, target = the pass's units
// spread over `budget` parts (at least kVMinPartUnits), so a slice that
// draws a large share of the lookups -- the last file of a level takes every
// key past the level's range (FindFile's quirk) -- is walked by many
// workgroups instead of one.  plan = exclusive prefix of the parts (S+1
// entries); the counters are zeroed for the next pass.
constexpr uint32_t kVMinPartUnits = 4096;
__global__ __launch_bounds__(1024) void version_plan_kernel(uint32_t* __restrict__ gcnt, uint32_t S, uint32_t budget,
                                                            uint32_t* __restrict__ plan) {
  __shared__ uint32_t a[kVMaxSlices + 1];
  __shared__ uint32_t wsum[16];
  __shared__ uint32_t tot;
  const int tid = threadIdx.x;
  uint32_t c = 0;
  if (static_cast<uint32_t>(tid) < S) {
    c = gcnt[tid];
    gcnt[tid] = 0;
  }
  const uint32_t sum = wave_sum(c);
  if ((tid & 63) == 0) wsum[tid >> 6] = sum;
  __syncthreads();
  if (tid == 0) {
    uint32_t t = 0;
    for (int w = 0; w < 16; w++) t += wsum[w];
    tot = t;
  }
  __syncthreads();
  const uint32_t target = max(kVMinPartUnits, (tot + budget - 1) / budget);
  if (static_cast<uint32_t>(tid) < S) a[tid] = max(1u, (c + target - 1) / target);
  if (tid == 0) a[S] = 0;
  __syncthreads();
  block_excl_scan_lds<1024>(a, static_cast<int>(S + 1), wsum);
  for (uint32_t b = tid; b <= S; b += 1024) plan[b] = a[b];
}

// Sliced version probe, unpermute (one workgroup per chunk): the chunk's
// answers (bit 0 of each answer byte, at the entries' positions) staged in
// LDS, then per lookup its answer -- 0 without a probe in this pass -- into
// abyte bit jbit (written by the first pass, OR-ed by later ones); the last
// pass folds every sliced level's bit into slot_mask at its slot.
__global__ __launch_bounds__(kBlock) void version_unpermute_kernel(uint64_t n, const uint16_t* __restrict__ pos,
                                                                   const uint8_t* __restrict__ smask,
                                                                   uint8_t* __restrict__ abyte,
                                                                   uint64_t* __restrict__ slot_mask, int jbit,
                                                                   int n_sliced, uint64_t slots, int first,
                                                                   int last) {
  __shared__ __attribute__((aligned(16))) uint8_t sm[kVRegion];
  const int tid = threadIdx.x;
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kVChunk;
  const uint32_t nk = static_cast<uint32_t>(min(static_cast<uint64_t>(kVChunk), n - base));
  const uint4* s4 = reinterpret_cast<const uint4*>(smask + static_cast<uint64_t>(blockIdx.x) * kVRegion);
  for (uint32_t v = tid; v < kVRegion / 16u; v += kBlock) reinterpret_cast<uint4*>(sm)[v] = s4[v];
  __syncthreads();
  for (uint32_t i = tid; i < nk; i += kBlock) {
    const uint16_t p = pos[base + i];
    const uint32_t bit = p == kVNoPos ? 0u : (sm[p] & 1u);
    uint32_t a = bit << jbit;
    if (!first) a |= abyte[base + i];
    if (!last) {
      abyte[base + i] = static_cast<uint8_t>(a);
      continue;
    }
    uint64_t m = slot_mask[base + i];
    for (int j = 0; j < n_sliced; j++) m |= static_cast<uint64_t>((a >> j) & 1u) << ((slots >> (8 * j)) & 63u);
    slot_mask[base + i] = m;
  }
}

// ---------------------------------------------------------------------------
// Legacy FilterPolicy format (util/bloom.cc): global double hashing.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t dec32_dev(const uint8_t* p) {  // DecodeFixed32, any alignment
  return static_cast<uint32_t>(p[0]) | (static_cast<uint32_t>(p[1]) << 8) |
         (static_cast<uint32_t>(p[2]) << 16) | (static_cast<uint32_t>(p[3]) << 24);
}

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

// ---------------------------------------------------------------------------
// Legacy FilterPolicy build, LDS-tiled (util/bloom.cc:25-55).  The legacy
// format spreads a key's k bits over the WHOLE filter (bitpos = h % bits,
// then h += rotr(h, 17)), so the unit the build buckets is one bit position,
// not one key.  Pass 1 (partition, one 512-thread workgroup per 4,096-key
// chunk): hash each key once, compute its k positions, and bucket them by
// 8 KiB tile (2^16 bits) as u16 offsets inside the tile -- 2k bytes per key;
// every bucket is padded to whole 16-byte units with copies of its first
// entry (setting a bit twice changes nothing).  Pass 2 (slice, one
// 1,024-thread workgroup per 2^TPS_LG consecutive tiles of one filter): the
// tiles live in LDS, every wave walks its share of the chunks (one contiguous
// run per chunk: the slice's buckets are adjacent), sets bits with ds_or and
// the tiles stream out with 16-byte stores.  No global atomics: the direct
// kernel's 6 device-scope atomicOr per key are memory-side operations on
// 64 random rows per wave instruction.
// ---------------------------------------------------------------------------
template <int MODE, int KMAX, uint32_t STAGE, uint32_t TMAX>
__global__ __launch_bounds__(kLegacyPartBlock) void legacy_partition_kernel(
    const LegacyTileJobDev* __restrict__ jobs, const uint32_t* __restrict__ chunk0s, int n_jobs,
    uint16_t* __restrict__ entries, uint16_t* __restrict__ tab) {
  constexpr int NT = kLegacyPartBlock;
  constexpr int C = kLegacyChunk;
  constexpr int PER = C / NT;
  constexpr int KB = mode_kb<MODE>();
  constexpr int TKV = K20Tile<NT, tile_kpt<KB>(), KB>::kVec;  // uint4 of one key tile
  constexpr int SV = static_cast<int>(STAGE / 8u);            // uint4 of one staged region
  constexpr int TVB = TKV > SV ? TKV : SV;
  static_assert(TMAX + 1 <= 4u * NT, "block_excl_scan_lds covers the tile bins");
  __shared__ __attribute__((aligned(16))) uint4 tile[TVB];
  __shared__ uint32_t hist[TMAX + 1];
  __shared__ uint8_t npad[TMAX];
  __shared__ uint32_t wsum[NT / 64];
  __shared__ int sj;
  const int tid = threadIdx.x;
  const uint32_t bid = blockIdx.x;
  if (tid == 0) sj = find_job(chunk0s, n_jobs, bid);
  __syncthreads();
  const LegacyTileJobDev J = jobs[sj];
  const uint32_t c = bid - J.chunk0;
  const uint64_t first = static_cast<uint64_t>(c) * C;
  const uint64_t left = J.keys.n - first;
  const uint32_t nk = left < static_cast<uint64_t>(C) ? static_cast<uint32_t>(left) : C;
  uint32_t h[PER];
  hash_chunk<MODE, NT, PER>(J.keys, first, nk, tile, h);
  const uint32_t nT = J.n_tiles, bits = J.bits, magic = J.magic;
  const int k = J.k;
  for (uint32_t b = tid; b <= nT; b += NT) hist[b] = 0;
  __syncthreads();
  // Count the positions per tile (the positions are computed twice -- here
  // and in the scatter -- rather than kept: 8 keys x k codes per thread would
  // hold ~50 more VGPRs and halve the workgroups per CU).
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const bool live = static_cast<uint32_t>(r * NT + tid) < nk;
    uint32_t hh = h[r];
    const uint32_t delta = bloom_delta(hh);
#pragma unroll
    for (int q = 0; q < KMAX; q++) {
      if (live && q < k) atomicAdd(&hist[fastmod(hh, bits, magic) >> kLegacyTileLg], 1u);
      hh += delta;
    }
  }
  __syncthreads();
  for (uint32_t b = tid; b < nT; b += NT) {  // pad every bucket to whole 16-byte units
    const uint32_t cnt = hist[b];
    const uint32_t pad = (0u - cnt) & 7u;
    npad[b] = static_cast<uint8_t>(pad);
    hist[b] = cnt + pad;
  }
  __syncthreads();
  const uint32_t total = block_excl_scan_lds<NT>(hist, static_cast<int>(nT + 1), wsum);
  uint16_t* trow = tab + J.tab0 + static_cast<uint64_t>(c) * (nT + 1);
  for (uint32_t b = tid; b <= nT; b += NT) trow[b] = static_cast<uint16_t>(hist[b]);
  uint16_t* stage = reinterpret_cast<uint16_t*>(tile);  // free since hash_chunk's last barrier
  __syncthreads();  // hist becomes the buckets' fill cursors
  // Scatter: a bucket's order is whatever the LDS atomics give -- the slice
  // pass ORs bits, so the order of a tile's positions never shows.
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const bool live = static_cast<uint32_t>(r * NT + tid) < nk;
    uint32_t hh = h[r];
    const uint32_t delta = bloom_delta(hh);
#pragma unroll
    for (int q = 0; q < KMAX; q++) {
      if (live && q < k) {
        const uint32_t bp = fastmod(hh, bits, magic);
        stage[atomicAdd(&hist[bp >> kLegacyTileLg], 1u)] = static_cast<uint16_t>(bp);
      }
      hh += delta;
    }
  }
  __syncthreads();
  for (uint32_t b = tid; b < nT; b += NT) {  // pads: copies of the bucket's last position
    const uint32_t np = npad[b];
    if (np) {
      const uint32_t end = hist[b];  // the cursor stopped after the last real position
      const uint16_t v = stage[end - 1];
      for (uint32_t p = 0; p < np; p++) stage[end + p] = v;
    }
  }
  __syncthreads();
  store_chunk_u16<NT>(entries + J.entry0 + static_cast<uint64_t>(c) * J.region, stage, total);
}

// One chunk's run of a legacy slice, as one wave sees it: lane j <= tn holds
// the table row's offset of tile t0 + j (u16 entries); r0 / T / the unit
// offsets of the tile starts are wave-uniform.
struct LegacyRun {
  uint32_t r0, T;           // first entry of the run, its length in 16-byte units
  uint32_t ts[15];          // unit offset of tile j + 1 inside the run (j < tn - 1)
  const uint4* base;
};

template <uint32_t TPS>
__device__ __forceinline__ LegacyRun legacy_run(uint32_t row, uint32_t tn, const uint16_t* ent,
                                                uint64_t region_off) {
  LegacyRun R;
  R.r0 = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(row), 0));
  const uint32_t rend = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(row), static_cast<int>(tn)));
  R.T = (rend - R.r0) >> 3;
#pragma unroll
  for (uint32_t j = 0; j + 1 < TPS; j++) {
    const uint32_t lj = min(j + 1u, tn);
    R.ts[j] = (static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(row), static_cast<int>(lj))) - R.r0) >> 3;
  }
  R.base = reinterpret_cast<const uint4*>(ent + region_off + R.r0);
  return R;
}

// OR the 8 positions of unit u (of run R) into the slice's LDS tiles.
template <uint32_t TPS>
__device__ __forceinline__ void legacy_or_unit(uint32_t* sl, const LegacyRun& R, uint32_t u, const uint4& v) {
  uint32_t m = 0;
#pragma unroll
  for (uint32_t j = 0; j + 1 < TPS; j++) m += u >= R.ts[j] ? 1u : 0u;  // tiles past tn repeat the run's end
  uint32_t* t = sl + (m << 11);
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t lo = w[q] & 0xffffu, hi = w[q] >> 16;
    atomicOr(&t[lo >> 5], 1u << (lo & 31u));
    atomicOr(&t[hi >> 5], 1u << (hi & 31u));
  }
}

template <int TPS_LG>
__global__ __launch_bounds__(kLegacySliceBlock) void legacy_slice_kernel(
    const LegacyTileJobDev* __restrict__ jobs, const uint32_t* __restrict__ slice0s, int n_jobs,
    const uint16_t* __restrict__ entries, const uint16_t* __restrict__ tab) {
  constexpr uint32_t TPS = 1u << TPS_LG;
  constexpr int NW = kLegacySliceBlock / 64;
  constexpr int UPL = 4;  // units in flight per lane per chunk (256 units = 2,048 positions)
  __shared__ __attribute__((aligned(16))) uint32_t sl[TPS * 2048u];
  __shared__ int sj;
  const int tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t wv = static_cast<uint32_t>(wave_id());
  const uint32_t bid = xcd_block(blockIdx.x, gridDim.x);
  if (tid == 0) sj = find_job(slice0s, n_jobs, bid);
  for (uint32_t w = tid; w < TPS * 512u; w += kLegacySliceBlock) reinterpret_cast<uint4*>(sl)[w] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  const LegacyTileJobDev J = jobs[sj];
  const uint32_t s = bid - J.slice0;
  const uint32_t t0 = s << TPS_LG;
  const uint32_t nT = J.n_tiles;
  const uint32_t tn = min(TPS, nT - t0);
  const uint32_t nC = J.n_chunks, rowlen = nT + 1;
  const uint16_t* tb = tab + J.tab0 + t0;
  const uint16_t* ent = entries + J.entry0;
  // Row loads are clamped (unconditional); a wave works chunk c while chunk
  // c + NW's row and units are already in flight.
  auto row_at = [&](uint32_t cc) -> uint32_t {
    const uint32_t c1 = min(cc, nC - 1u);
    return tb[static_cast<uint64_t>(c1) * rowlen + min(lane, tn)];
  };
  auto fetch = [&](const LegacyRun& R, uint4 (&v)[UPL]) {
#pragma unroll
    for (int i = 0; i < UPL; i++) {
      const uint32_t u = min(lane + 64u * i, R.T - 1u);  // T > 0 when fetched
      v[i] = R.base[u];
    }
  };
  auto consume = [&](const LegacyRun& R, const uint4 (&v)[UPL]) {
#pragma unroll
    for (int i = 0; i < UPL; i++) {
      const uint32_t u = lane + 64u * i;
      if (u < R.T) legacy_or_unit<TPS>(sl, R, u, v[i]);
    }
    for (uint32_t u = lane + 64u * UPL; u < R.T; u += 64u) legacy_or_unit<TPS>(sl, R, u, R.base[u]);  // long runs
  };
  uint32_t c = wv;
  if (c < nC) {
    uint32_t rowA = row_at(c);
    uint32_t rowN = row_at(c + NW);
    LegacyRun A = legacy_run<TPS>(rowA, tn, ent, static_cast<uint64_t>(c) * J.region);
    uint4 vA[UPL];
    if (A.T) fetch(A, vA);
    while (true) {
      const uint32_t cn = c + NW;
      const bool more = cn < nC;
      LegacyRun B;
      uint4 vB[UPL];
      if (more) {
        B = legacy_run<TPS>(rowN, tn, ent, static_cast<uint64_t>(cn) * J.region);
        if (B.T) fetch(B, vB);
        rowN = row_at(cn + NW);
      }
      if (A.T) consume(A, vA);
      if (!more) break;
      A = B;
#pragma unroll
      for (int i = 0; i < UPL; i++) vA[i] = vB[i];
      c = cn;
    }
  }
  __syncthreads();
  // Stream the tiles out: bytes [t0 * 8 KiB, min((t0 + tn) * 8 KiB, bits / 8)).
  const uint64_t bytes = J.bits / 8u;
  const uint64_t b0 = static_cast<uint64_t>(t0) << (kLegacyTileLg - 3);
  const uint64_t nb = min(static_cast<uint64_t>(tn) << (kLegacyTileLg - 3), bytes - b0);
  uint8_t* dst = J.out + b0;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(sl);
  if ((reinterpret_cast<uintptr_t>(J.out) & 15u) == 0) {
    const uint32_t nv = static_cast<uint32_t>(nb >> 4);
    for (uint32_t w = tid; w < nv; w += kLegacySliceBlock)
      st_global16(reinterpret_cast<uint4*>(dst) + w, reinterpret_cast<const uint4*>(src)[w]);
    for (uint32_t i = nv * 16u + tid; i < nb; i += kLegacySliceBlock) st_global1(dst + i, src[i]);
  } else {
    for (uint32_t i = tid; i < nb; i += kLegacySliceBlock) st_global1(dst + i, src[i]);
  }
  if (s == 0 && tid == 0) {
    J.out[bytes] = static_cast<uint8_t>(static_cast<int8_t>(J.k));  // dst->append(&hash_num, 1)
    *J.out_len = bytes + 1u;
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
                             uint32_t total_chunks, uint32_t* dchunk, int mode, hipStream_t s) {
  if (total_chunks == 0) return hipSuccess;
  if (mode == KM_K20)
    full_partition_kernel<KM_K20, false><<<total_chunks, kPartBlock, 0, s>>>(jobs, chunk0s, n_jobs, dchunk,
                                                                          nullptr, nullptr, 0, 0u);
  else if (mode == KM_HASH)
    full_partition_kernel<KM_HASH, false><<<total_chunks, kPartBlock, 0, s>>>(jobs, chunk0s, n_jobs, dchunk,
                                                                           nullptr, nullptr, 0, 0u);
  else if (mode == KM_K28)
    full_partition_kernel<KM_K28, false><<<total_chunks, kPartBlock, 0, s>>>(jobs, chunk0s, n_jobs, dchunk,
                                                                          nullptr, nullptr, 0, 0u);
  else
    full_partition_kernel<KM_GENERIC, false><<<total_chunks, kPartBlock, 0, s>>>(
        jobs, chunk0s, n_jobs, dchunk, nullptr, nullptr, 0, 0u);
  return hipGetLastError();
}

hipError_t launch_full_zero(const FullJobDev* jobs, int n_jobs, const uint32_t* dchunk,
                            uint32_t* jobL, hipStream_t s) {
  if (n_jobs == 0) return hipSuccess;
  full_zero_kernel<<<dim3(64, n_jobs), kBlock, 0, s>>>(jobs, dchunk, jobL);
  return hipGetLastError();
}

hipError_t launch_full_scatter(const FullJobDev* jobs, const uint32_t* chunk0s, int n_jobs,
                               uint32_t total_chunks, const uint32_t* jobL, int mode, hipStream_t s) {
  if (total_chunks == 0) return hipSuccess;
  if (mode == KM_K20)
    full_scatter_kernel<KM_K20><<<total_chunks, kBlock, 0, s>>>(jobs, chunk0s, n_jobs, jobL);
  else if (mode == KM_HASH)
    full_scatter_kernel<KM_HASH><<<total_chunks, kBlock, 0, s>>>(jobs, chunk0s, n_jobs, jobL);
  else
    full_scatter_kernel<KM_GENERIC><<<total_chunks, kBlock, 0, s>>>(jobs, chunk0s, n_jobs, jobL);
  return hipGetLastError();
}

hipError_t launch_full_partition(const FullJobDev* jobs, const uint32_t* chunk0s, int n_jobs,
                                 uint32_t chunk_first, uint32_t n_chunks, uint32_t* dchunk,
                                 uint32_t* entries, uint16_t* tab, int lgR, int mode, bool exact,
                                 hipStream_t s) {
  if (n_chunks == 0) return hipSuccess;
#define DLSM_PART(MM, EX)                                                                   \
  full_partition_kernel<MM, true, EX><<<n_chunks, kPartBlock, 0, s>>>(jobs, chunk0s, n_jobs, \
                                                                      dchunk, entries, tab, lgR, chunk_first)
  if (mode == KM_K20) {
    if (exact) DLSM_PART(KM_K20, true); else DLSM_PART(KM_K20, false);
  } else if (mode == KM_HASH) {
    DLSM_PART(KM_HASH, true);  // hashed jobs always run the count pass first
  } else if (mode == KM_K28) {
    if (exact) DLSM_PART(KM_K28, true); else DLSM_PART(KM_K28, false);
  } else {
    if (exact) DLSM_PART(KM_GENERIC, true); else DLSM_PART(KM_GENERIC, false);
  }
#undef DLSM_PART
  return hipGetLastError();
}

hipError_t launch_full_slices(const FullJobDev* jobs, const uint32_t* slice0s, int n_jobs,
                              uint32_t slice_first, uint32_t n_slices, const uint32_t* dchunk,
                              const uint32_t* entries, const uint16_t* tab, int lgR, hipStream_t s,
                              uint32_t* crc_part, const uint32_t* crc_tabs, uint32_t* crc_cnt) {
  if (n_slices == 0) return hipSuccess;
#define DLSM_FSL(LG)                                                                                          \
  do {                                                                                                        \
    if (crc_part)                                                                                             \
      full_slice_kernel<LG, true><<<n_slices, kSliceBlock, 0, s>>>(jobs, slice0s, n_jobs, dchunk, entries, tab, \
                                                                   slice_first, crc_part, crc_tabs, crc_cnt);\
    else                                                                                                      \
      full_slice_kernel<LG, false><<<n_slices, kSliceBlock, 0, s>>>(jobs, slice0s, n_jobs, dchunk, entries,     \
                                                                    tab, slice_first);                       \
  } while (0)
  switch (lgR) {
    case 7: DLSM_FSL(7); break;
    case 8: DLSM_FSL(8); break;
    case 9: DLSM_FSL(9); break;
    case 10: DLSM_FSL(10); break;
    case 11: DLSM_FSL(11); break;
    default: return hipErrorInvalidValue;
  }
#undef DLSM_FSL
  return hipGetLastError();
}

hipError_t launch_full_block_seal(const FullJobDev* jobs, int n_jobs, const uint32_t* crc_part,
                                  const uint32_t* crc_tabs, int lgR, hipStream_t s) {
  if (n_jobs == 0 || DLSM_SEAL_LAST) return hipSuccess;  // the slices sealed the filters
  switch (lgR) {
    case 7: full_block_seal_kernel<7><<<n_jobs, 256, 0, s>>>(jobs, crc_part, crc_tabs); break;
    case 8: full_block_seal_kernel<8><<<n_jobs, 256, 0, s>>>(jobs, crc_part, crc_tabs); break;
    case 9: full_block_seal_kernel<9><<<n_jobs, 256, 0, s>>>(jobs, crc_part, crc_tabs); break;
    case 10: full_block_seal_kernel<10><<<n_jobs, 256, 0, s>>>(jobs, crc_part, crc_tabs); break;
    case 11: full_block_seal_kernel<11><<<n_jobs, 256, 0, s>>>(jobs, crc_part, crc_tabs); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_probe_direct(const FilterDev* fs, int n_filters, KeyDesc keys, uint8_t* mask,
                               int mode, hipStream_t s) {
  if (keys.n == 0) return hipSuccess;
  const unsigned g = grid_for(keys.n, 256u * 64u);
  if (mode == KM_K20)
    probe_direct_kernel<KM_K20><<<g, kBlock, 0, s>>>(fs, n_filters, keys, mask);
  else if (mode == KM_HASH)
    probe_direct_kernel<KM_HASH><<<g, kBlock, 0, s>>>(fs, n_filters, keys, mask);
  else
    probe_direct_kernel<KM_GENERIC><<<g, kBlock, 0, s>>>(fs, n_filters, keys, mask);
  return hipGetLastError();
}

__global__ __launch_bounds__(kBlock) void probe_direct_group_kernel(const FilterDev* __restrict__ slots,
                                                                    KeyDesc hk, uint8_t* __restrict__ mask,
                                                                    int stride, int byte, int first) {
  __shared__ FilterDev sf[8];
  if (threadIdx.x < 8) sf[threadIdx.x] = slots[threadIdx.x];
  __syncthreads();
  const uint32_t* hv = reinterpret_cast<const uint32_t*>(hk.bytes);
  for (uint64_t i = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x; i < hk.n;
       i += static_cast<uint64_t>(gridDim.x) * kBlock) {
    const uint32_t h = hv[i];
    uint32_t m = 0;
#pragma unroll
    for (int b = 0; b < 8; b++)
      if (sf[b].data) m |= full_may_match(h, sf[b]) << b;
    uint8_t* o = mask + i * static_cast<uint64_t>(stride) + byte;
    *o = first ? static_cast<uint8_t>(m) : static_cast<uint8_t>(*o | m);
  }
}

hipError_t launch_probe_direct_group(const FilterDev* slots, KeyDesc hashes, uint8_t* mask, int stride,
                                     int byte, bool first, hipStream_t s) {
  if (hashes.n == 0) return hipSuccess;
  probe_direct_group_kernel<<<grid_for(hashes.n, 256u * 64u), kBlock, 0, s>>>(slots, hashes, mask, stride,
                                                                              byte, first);
  return hipGetLastError();
}

hipError_t launch_stack_filters(const FilterDev* slots, uint32_t L, uint64_t* stacked, hipStream_t s) {
  const uint64_t words = static_cast<uint64_t>(L) * 64u;
  stack_filters_kernel<<<grid_for(words), kBlock, 0, s>>>(slots, words, stacked);
  return hipGetLastError();
}

// Packed image of 1, 2 or up to 4 filters (W = 2^lgw bits per bit position):
// bit m of field p of line l = bit p of line l of member m (the filter's own
// layout: byte p >> 3, bit p & 7, util/bloom_impl.h:427-443).  W = 1 is the
// filter's bytes unchanged.  One u64 word (64 / W positions) per thread; the
// image is built once per filter set.
__global__ __launch_bounds__(kBlock) void pack_filters_kernel(const FilterDev* __restrict__ slots,
                                                              uint32_t slotmap, int lgw, uint64_t words,
                                                              uint64_t* __restrict__ packed) {
  const int W = 1 << lgw;
  const uint8_t* src[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int m = 0; m < W; m++) src[m] = slots[(slotmap >> (4 * m)) & 7u].data;
  const uint64_t per_line = 8u << lgw;  // u64 words per line (64 * W bytes)
  for (uint64_t w = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x; w < words;
       w += static_cast<uint64_t>(gridDim.x) * kBlock) {
    const uint64_t line = w / per_line;
    const uint32_t p0 = static_cast<uint32_t>(w % per_line) * (64u >> lgw);  // first position of the word
    uint64_t x = 0;
    for (int m = 0; m < W; m++) {
      if (!src[m]) continue;
      const uint8_t* ln = src[m] + line * 64u;
      for (uint32_t i = 0; i < (64u >> lgw); i++) {
        const uint32_t pp = p0 + i;
        x |= static_cast<uint64_t>((ln[pp >> 3] >> (pp & 7u)) & 1u) << ((i << lgw) + m);
      }
    }
    packed[w] = x;
  }
}

hipError_t launch_pack_filters(const FilterDev* slots, uint32_t slotmap, int lgw, uint32_t L,
                               uint64_t* packed, hipStream_t s) {
  if (lgw < 0 || lgw > 2) return hipErrorInvalidValue;
  const uint64_t words = static_cast<uint64_t>(L) * (8u << lgw);
  pack_filters_kernel<<<grid_for(words), kBlock, 0, s>>>(slots, slotmap, lgw, words, packed);
  return hipGetLastError();
}

// Hash pass of the grouped probe: one 512-thread workgroup per 4,096 keys,
// the key tiles staged through LDS like the partition's (K20 / K28), the
// hashes stored coalesced.
template <int MODE>
__global__ __launch_bounds__(512) void probe_hash_kernel(KeyDesc kd, uint32_t* __restrict__ hashes) {
  constexpr int NT = 512, C = 4096, PER = C / NT;
  constexpr int KB = mode_kb<MODE>();
  constexpr int TV = K20Tile<NT, tile_kpt<KB>(), KB>::kVec;
  __shared__ __attribute__((aligned(16))) uint4 tile[TV];
  const uint64_t first = static_cast<uint64_t>(blockIdx.x) * C;
  const uint64_t left = kd.n - first;
  const uint32_t nk = left < static_cast<uint64_t>(C) ? static_cast<uint32_t>(left) : C;
  uint32_t h[PER];
  hash_chunk<MODE, NT, PER>(kd, first, nk, tile, h);
#pragma unroll
  for (int r = 0; r < PER; r++) {
    const uint32_t i = r * NT + threadIdx.x;
    if (i < nk) hashes[first + i] = h[r];
  }
}

hipError_t launch_probe_hash(KeyDesc keys, uint32_t* hashes, int mode, hipStream_t s) {
  if (keys.n == 0) return hipSuccess;
  const unsigned g = static_cast<unsigned>((keys.n + 4095) / 4096);
  if (mode == KM_K20)
    probe_hash_kernel<KM_K20><<<g, 512, 0, s>>>(keys, hashes);
  else if (mode == KM_K28)
    probe_hash_kernel<KM_K28><<<g, 512, 0, s>>>(keys, hashes);
  else
    probe_hash_kernel<KM_GENERIC><<<g, 512, 0, s>>>(keys, hashes);
  return hipGetLastError();
}

// Compute units of the current device (cached per device id; builder threads
// call this concurrently, so the cache is atomic).
static uint32_t device_cus() {
  static std::atomic<uint32_t> cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256u;
  uint32_t c = cus[dev].load(std::memory_order_relaxed);
  if (!c) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    c = static_cast<uint32_t>(n);
    cus[dev].store(c, std::memory_order_relaxed);
  }
  return c;
}

// Largest LDS allocation of one workgroup on device `dev` (cached per device
// id like device_cus).
static size_t device_lds_max(int dev) {
  static std::atomic<uint32_t> lds[64] = {};
  if (dev < 0 || dev >= 64) return 64u * 1024u;
  uint32_t c = lds[dev].load(std::memory_order_relaxed);
  if (!c) {
    // the opt-in ceiling (what hipFuncAttributeMaxDynamicSharedMemorySize may
    // raise a kernel to), else the default per-block one
    int a = 0, b = 0;
    if (hipDeviceGetAttribute(&a, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess) a = 0;
    if (hipDeviceGetAttribute(&b, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess) b = 0;
    const int n = std::max(std::max(a, b), 64 * 1024);
    c = static_cast<uint32_t>(n);
    lds[dev].store(c, std::memory_order_relaxed);
  }
  return c;
}

#ifndef DLSM_PROBE_P13_HALF
#define DLSM_PROBE_P13_HALF 1
#endif
#ifndef DLSM_PROBE_UNITS14
#define DLSM_PROBE_UNITS14 2
#endif
// Probe chunk shapes: C keys per partition workgroup of NT threads.
//   lgC 12: C = 4096, 512 threads;  13: 8192, 1024;  14: 16384, 1024.
template <int C, int NT, int H = 1>
static hipError_t probe_partition_as(KeyDesc keys, uint32_t L, uint32_t magic, uint32_t R,
                                     uint32_t n_slices, uint32_t* entries, uint16_t* pos,
                                     uint16_t* tab, int mode, hipStream_t s, uint32_t cus) {
  const uint32_t nC = static_cast<uint32_t>((keys.n + C - 1) / C);
  if (nC == 0) return hipSuccess;
  // One workgroup per chunk (default), or persistent: $DLSM_PART_GRID_PER_CU
  // resident workgroups per CU looping over the chunks with the next chunk's
  // key tiles in flight.  Round 4 (`profiles/r04_o_grid0_shares_ab.txt`): one
  // workgroup per chunk takes the probe pass 0.685 -> 0.645 ms and the
  // overlapped step -4 % (the hardware's dispatcher keeps every CU's phases
  // mixed, with no tail of long-running workgroups and room for the build's
  // workgroups beside them); neutral at the N = 4 / 8 shares.
  // Only 20-byte keys take one workgroup per chunk by default: 28-byte
  // internal keys (their one-per-chunk form spills more: 6 % slower,
  // `profiles/r04_z_internal_keys_grid_ab.txt`) and hashed lookups (4 %
  // slower, `r04_z4_hashed_probe_grid_ab.txt`) keep the persistent grid, as
  // do variable-length keys (round 3's default, not re-measured).
  static const int per_cu_env = [] {
    const char* e = getenv("DLSM_PART_GRID_PER_CU");
    return e ? atoi(e) : -1;
  }();
  const uint32_t per_cu = per_cu_env >= 0 ? static_cast<uint32_t>(per_cu_env) : (mode == KM_K20 ? 0u : 2u);
  const uint32_t g = per_cu ? std::min(nC, per_cu * (cus ? cus : device_cus())) : nC;
  // $DLSM_PROBE_PLAIN_STORES=1: plain (Infinity-Cache-allocating) intermediate
  // stores, for round-sized batches (A/B knob; K20 keys only)
  static const bool plain = [] {
    const char* e = getenv("DLSM_PROBE_PLAIN_STORES");
    return e && atoi(e) != 0;
  }();
#ifndef DLSM_PPART_PERSIST_ALWAYS
#define DLSM_PPART_PERSIST_ALWAYS 0  // A/B: the persistent instantiation at every grid size
#endif
#define DLSM_PPART(MM, NTS_)                                                                                   \
  do {                                                                                                         \
    if (per_cu || DLSM_PPART_PERSIST_ALWAYS)                                                                   \
      probe_partition_kernel<MM, NT, C, H, NTS_, true><<<g, NT, 0, s>>>(keys, L, magic, R, fastmod_magic(R),  \
                                                                        n_slices, nC, entries, pos, tab);      \
    else                                                                                                       \
      probe_partition_kernel<MM, NT, C, H, NTS_, false><<<g, NT, 0, s>>>(keys, L, magic, R, fastmod_magic(R), \
                                                                         n_slices, nC, entries, pos, tab);     \
  } while (0)
  if (mode == KM_HASH)
    DLSM_PPART(KM_HASH, true);
  else if (mode == KM_K20 && plain)
    DLSM_PPART(KM_K20, false);
  else if (mode == KM_K20)
    DLSM_PPART(KM_K20, true);
  else if (mode == KM_K28)
    DLSM_PPART(KM_K28, true);
  else
    DLSM_PPART(KM_GENERIC, true);
#undef DLSM_PPART
  return hipGetLastError();
}

hipError_t launch_probe_partition(KeyDesc keys, uint32_t L, uint32_t magic, uint32_t R,
                                  uint32_t n_slices, uint32_t* entries, uint16_t* pos,
                                  uint16_t* tab, int mode, int lgC, hipStream_t s, uint32_t cus) {
  switch (lgC) {
    case 12: return probe_partition_as<4096, 512>(keys, L, magic, R, n_slices, entries, pos, tab, mode, s, cus);
#if DLSM_PROBE_P13_HALF
    // 512-thread workgroups of two 4,096-key units (two resident per CU)
    case 13: return probe_partition_as<8192, 512, 2>(keys, L, magic, R, n_slices, entries, pos, tab, mode, s, cus);
#else
    case 13: return probe_partition_as<8192, 1024>(keys, L, magic, R, n_slices, entries, pos, tab, mode, s, cus);
#endif
    // 16,384-key chunks bucketed as two 8,192-key units (DLSM_PROBE_UNITS14)
    case 14: return probe_partition_as<16384, 1024, DLSM_PROBE_UNITS14>(keys, L, magic, R, n_slices, entries, pos, tab, mode, s, cus);
    default: return hipErrorInvalidValue;
  }
}

template <int LGR, int LGW, int C>
static hipError_t probe_slices_as(const uint64_t* stacked, uint32_t L, uint32_t R, uint32_t slotmap, int k,
                                  uint32_t n_slices, uint32_t n_chunks, const uint32_t* entries,
                                  const uint16_t* tab, uint8_t* smask, int parts, hipStream_t s) {
  const uint8_t* st = reinterpret_cast<const uint8_t*>(stacked);
  constexpr int NT = DLSM_PROBE_NT;
  if (R == 0 || R > (1u << LGR)) return hipErrorInvalidValue;
  if (k == 6)  // bits_per_key 10 (ChooseNumProbes)
    probe_slice_kernel<LGR, LGW, 6, NT, C><<<n_slices * parts, NT, 0, s>>>(
        st, L, R, slotmap, k, n_slices, n_chunks, entries, tab, smask, parts);
  else
    probe_slice_kernel<LGR, LGW, 0, NT, C><<<n_slices * parts, NT, 0, s>>>(
        st, L, R, slotmap, k, n_slices, n_chunks, entries, tab, smask, parts);
  return hipGetLastError();
}

hipError_t launch_probe_slices(const uint64_t* stacked, uint32_t L, uint32_t magic, int k, int lgR, uint32_t R,
                               int lgw, uint32_t slotmap, uint32_t n_slices, uint32_t n_chunks,
                               const uint32_t* entries, const uint16_t* tab, uint8_t* smask, int parts,
                               int lgC, hipStream_t s) {
  (void)magic;  // the partition already reduced every hash to its slice and line
  if (n_chunks == 0) return hipSuccess;
#define DLSM_SLICES(LG, LW, CC) \
  return probe_slices_as<LG, LW, CC>(stacked, L, R, slotmap, k, n_slices, n_chunks, entries, tab, smask, parts, s)
#define DLSM_SLICES_C(LG, LW)                  \
  do {                                         \
    if (lgC == 12) DLSM_SLICES(LG, LW, 4096);  \
    if (lgC == 13) DLSM_SLICES(LG, LW, 8192);  \
    if (lgC == 14) DLSM_SLICES(LG, LW, 16384); \
  } while (0)
  if (lgw == 3 && lgR == 7) DLSM_SLICES_C(7, 3);
  if (lgw == 3 && lgR == 8) DLSM_SLICES_C(8, 3);
  if (lgw == 2 && lgR == 9) DLSM_SLICES_C(9, 2);
  if (lgw == 1 && lgR == 10) DLSM_SLICES_C(10, 1);
  if (lgw == 0 && lgR == 11) DLSM_SLICES_C(11, 0);
#undef DLSM_SLICES_C
#undef DLSM_SLICES
  return hipErrorInvalidValue;
}

hipError_t launch_probe_unpermute(uint64_t n_keys, const uint16_t* pos, const uint8_t* smask,
                                  uint8_t* mask, int lgC, hipStream_t s) {
  if (n_keys == 0) return hipSuccess;
  const unsigned nC = static_cast<unsigned>((n_keys + (1ull << lgC) - 1) >> lgC);
  const bool vec = (reinterpret_cast<uintptr_t>(mask) & 7u) == 0;
#define DLSM_UNPERMUTE(CC)                                                         \
  if (vec) probe_unpermute_kernel<CC, true><<<nC, kBlock, 0, s>>>(n_keys, pos, smask, mask); \
  else probe_unpermute_kernel<CC, false><<<nC, kBlock, 0, s>>>(n_keys, pos, smask, mask)
  switch (lgC) {
    case 12: DLSM_UNPERMUTE(4096); break;
    case 13: DLSM_UNPERMUTE(8192); break;
    case 14: DLSM_UNPERMUTE(16384); break;
    default: return hipErrorInvalidValue;
  }
#undef DLSM_UNPERMUTE
  return hipGetLastError();
}

// Grouped-probe unpermute: like probe_unpermute_kernel, but the answer byte
// goes to byte `byte` of the key's `stride`-byte mask entry, OR-ed into it
// unless this is the first group of that byte.
template <int C, int VEC>
__global__ __launch_bounds__(kBlock) void probe_unpermute_group_kernel(
    uint64_t n, const uint16_t* __restrict__ pos, const uint8_t* __restrict__ smask,
    uint8_t* __restrict__ mask, int stride, int byte, int first_group) {
  constexpr uint32_t CR = probe_region(C);
  __shared__ __attribute__((aligned(16))) uint8_t sm[CR];
  const int tid = threadIdx.x;
  const uint64_t first = static_cast<uint64_t>(blockIdx.x) * C;
  const uint64_t left = n - first;
  const uint32_t nk = left < static_cast<uint64_t>(C) ? static_cast<uint32_t>(left) : C;
  const uint32_t nvec = (min(CR, nk + 4u * kMaxSlices) + 15u) / 16u;
  const uint4* s4 = reinterpret_cast<const uint4*>(smask + static_cast<uint64_t>(blockIdx.x) * CR);
  for (uint32_t v = tid; v < nvec; v += kBlock) reinterpret_cast<uint4*>(sm)[v] = s4[v];
  __syncthreads();
  // 8 keys per thread: one 16-byte load of their positions; VEC = 1 (one
  // mask byte per key) / 2 (two: 9..16 filters), mask aligned to 8 VEC bytes:
  // one 8- / 16-byte read-modify-write of their mask bytes; VEC = 0: byte
  // accesses at the group's byte of each key's stride.
  for (uint32_t i0 = 8u * tid; i0 < nk; i0 += 8u * kBlock) {
    if (i0 + 8u <= nk) {
      const uint4 pv = load_pos8(pos + first + i0);
      const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int q = 0; q < 2; q++) {
        lo |= uint32_t(sm[pw[q] & 0xffffu]) << (16 * q);
        lo |= uint32_t(sm[pw[q] >> 16]) << (16 * q + 8);
        hi |= uint32_t(sm[pw[q + 2] & 0xffffu]) << (16 * q);
        hi |= uint32_t(sm[pw[q + 2] >> 16]) << (16 * q + 8);
      }
      if constexpr (VEC == 1) {
        uint2* o = reinterpret_cast<uint2*>(mask + first + i0);
        if (!first_group) {
          const uint2 m = *o;
          lo |= m.x;
          hi |= m.y;
        }
        *o = make_uint2(lo, hi);
      } else if constexpr (VEC == 2) {
        // key b's two mask bytes are the 16-bit lane b; the group owns byte `byte` of each
        uint4* o = reinterpret_cast<uint4*>(mask + (first + i0) * 2u);
        const uint32_t sh = 8u * static_cast<uint32_t>(byte);
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint32_t src = q < 2 ? lo : hi;
          const uint32_t a0 = (src >> (16 * (q & 1))) & 0xffu, a1 = (src >> (16 * (q & 1) + 8)) & 0xffu;
          w[q] = (a0 << sh) | (a1 << (16u + sh));
        }
        uint4 m = make_uint4(w[0], w[1], w[2], w[3]);
        if (!first_group) {
          const uint4 old = *o;
          m.x |= old.x;
          m.y |= old.y;
          m.z |= old.z;
          m.w |= old.w;
        } else {
          // the first group of this byte writes it; keep the other byte
          const uint4 old = *o;
          const uint32_t keep = ~((0xffu << sh) | (0xffu << (16u + sh)));
          m.x |= old.x & keep;
          m.y |= old.y & keep;
          m.z |= old.z & keep;
          m.w |= old.w & keep;
        }
        *o = m;
      } else {
#pragma unroll
        for (int b = 0; b < 8; b++) {
          uint8_t* o = mask + (first + i0 + b) * static_cast<uint64_t>(stride) + byte;
          const uint8_t a = static_cast<uint8_t>((b < 4 ? lo : hi) >> (8 * (b & 3)));
          *o = first_group ? a : static_cast<uint8_t>(*o | a);
        }
      }
    } else {
      for (uint32_t i = i0; i < nk; i++) {
        uint8_t* o = mask + (first + i) * static_cast<uint64_t>(stride) + byte;
        const uint8_t a = sm[pos[first + i]];
        *o = first_group ? a : static_cast<uint8_t>(*o | a);
      }
    }
  }
}

hipError_t launch_probe_unpermute_group(uint64_t n_keys, const uint16_t* pos, const uint8_t* smask,
                                        uint8_t* mask, int stride, int byte, bool first, int lgC,
                                        hipStream_t s) {
  if (n_keys == 0) return hipSuccess;
  const unsigned nC = static_cast<unsigned>((n_keys + (1ull << lgC) - 1) >> lgC);
  const uintptr_t a = reinterpret_cast<uintptr_t>(mask);
  const int vec = (stride == 1 && (a & 7u) == 0) ? 1 : (stride == 2 && (a & 15u) == 0) ? 2 : 0;
#define DLSM_UNPERM_G(CC)                                                                                       \
  (vec == 1   ? (probe_unpermute_group_kernel<CC, 1><<<nC, kBlock, 0, s>>>(n_keys, pos, smask, mask, stride, byte, first), 0) \
   : vec == 2 ? (probe_unpermute_group_kernel<CC, 2><<<nC, kBlock, 0, s>>>(n_keys, pos, smask, mask, stride, byte, first), 0) \
              : (probe_unpermute_group_kernel<CC, 0><<<nC, kBlock, 0, s>>>(n_keys, pos, smask, mask, stride, byte, first), 0))
  switch (lgC) {
    case 12: DLSM_UNPERM_G(4096); break;
    case 13: DLSM_UNPERM_G(8192); break;
    case 14: DLSM_UNPERM_G(16384); break;
    default: return hipErrorInvalidValue;
  }
#undef DLSM_UNPERM_G
  return hipGetLastError();
}

// ---- one-pass multi-group probe launchers ----------------------------------
#ifndef DLSM_MG_NT
#define DLSM_MG_NT 256  // partition threads per 2,048-key chunk
#endif

// Dynamic LDS of the one-pass partition: the key tiles or the largest set's
// staged runs (stage_bytes, mg_layout), whichever is larger.
template <int MODE, int NT, int C>
static size_t mg_part_lds(uint32_t stage_bytes) {
  constexpr int KB = MODE == KM_K28 ? 28 : 20;
  using TL = K20Tile<NT, KB == 20 ? kTileKPT : 1, KB>;
  return std::max<size_t>(static_cast<size_t>(TL::kVec) * 16u, stage_bytes);
}

hipError_t launch_probe_mpartition(KeyDesc keys, const MGroupDev* groups, int G, uint32_t rowlen,
                                   uint32_t region, uint32_t stage_bytes, uint32_t* entries, uint16_t* pos,
                                   uint16_t* tab, int mode, hipStream_t s) {
  if (keys.n == 0) return hipSuccess;
  if (stage_bytes > 64u * 1024u) return hipErrorInvalidValue;
  if (G < 1 || G > kMGMaxGroups || rowlen > kMGMaxSlices + kMGMaxGroups || region > 65535u ||
      region % kMGPad != 0)
    return hipErrorInvalidValue;
  const int lgC = mg_chunk_lg(G);
  const uint64_t nC64 = (keys.n + (1ull << lgC) - 1) >> lgC;
  if (nC64 > 0xffffffffull) return hipErrorInvalidValue;
  const unsigned nC = static_cast<unsigned>(nC64);
#define DLSM_MPART(MM, NT_, C_, P_)                                                                            \
  probe_mpartition_kernel<MM, NT_, C_, P_><<<nC, NT_, mg_part_lds<MM, NT_, C_>(stage_bytes), s>>>(               \
      keys, groups, G, rowlen, region, entries, pos, tab)
#define DLSM_MPART_C(NT_, C_, P_)                               \
  do {                                                          \
    if (mode == KM_K20) DLSM_MPART(KM_K20, NT_, C_, P_);        \
    else if (mode == KM_K28) DLSM_MPART(KM_K28, NT_, C_, P_);   \
    else if (mode == KM_HASH) DLSM_MPART(KM_HASH, NT_, C_, P_); \
    else DLSM_MPART(KM_GENERIC, NT_, C_, P_);                   \
  } while (0)
  // (shapes: bloom_internal.h mg_chunk_lg; A/B knobs DLSM_MG_NT / DLSM_MG_P)
  if (lgC == 12) DLSM_MPART_C(512, 4096, 2);
  else if (lgC == 11) DLSM_MPART_C(DLSM_MG_NT, 2048, mg_set_size(11));
  else return hipErrorInvalidValue;
#undef DLSM_MPART_C
#undef DLSM_MPART
  return hipGetLastError();
}

template <int LGW, int K>
static hipError_t probe_mslices_as(const MGroupDev* groups, int G, uint32_t s0, uint32_t S, uint32_t rowlen,
                                   uint32_t region, uint32_t abytes, uint32_t n_chunks, const uint32_t* entries,
                                   const uint16_t* tab, uint8_t* answers, const uint32_t* plan, uint32_t wgs,
                                   hipStream_t s) {
  constexpr int NT = DLSM_PROBE_NT;
  probe_slice_kernel<11 - LGW, LGW, K, NT, 0, 0u, true><<<wgs, NT, 0, s>>>(
      nullptr, 0u, 0u, 0u, 0, S, n_chunks, entries, tab, answers, 1, plan, groups, G, s0, rowlen, region, abytes);
  return hipGetLastError();
}

hipError_t launch_probe_mslices(int lgw, int K, const MGroupDev* groups, int G, uint32_t s0, uint32_t S,
                                uint32_t rowlen, uint32_t region, uint32_t abytes, uint32_t n_chunks,
                                const uint32_t* entries, const uint16_t* tab, uint8_t* answers,
                                const uint32_t* plan, uint32_t wgs, hipStream_t s) {
  if (n_chunks == 0 || S == 0 || wgs == 0) return hipSuccess;
  if (region % kMGPad != 0 || abytes % 16u != 0 || (K != 0 && K != 6)) return hipErrorInvalidValue;
#define DLSM_MSL(LW)                                                                                          \
  return K == 6 ? probe_mslices_as<LW, 6>(groups, G, s0, S, rowlen, region, abytes, n_chunks, entries, tab, \
                                          answers, plan, wgs, s)                                            \
                : probe_mslices_as<LW, 0>(groups, G, s0, S, rowlen, region, abytes, n_chunks, entries, tab, \
                                          answers, plan, wgs, s)
  switch (lgw) {
    case 0: DLSM_MSL(0);
    case 1: DLSM_MSL(1);
    case 2: DLSM_MSL(2);
    case 3: DLSM_MSL(3);
    default: return hipErrorInvalidValue;
  }
#undef DLSM_MSL
}

hipError_t launch_probe_munpermute(uint64_t n_keys, const MGroupDev* groups, int G, uint32_t abytes,
                                   const uint16_t* pos, const uint8_t* answers, uint8_t* mask, int mask_bytes,
                                   hipStream_t s) {
  if (n_keys == 0) return hipSuccess;
  if (mask_bytes < 1 || mask_bytes > 8 || abytes % 16u != 0 || abytes > 96u * 1024u) return hipErrorInvalidValue;
  const int lgC = mg_chunk_lg(G);
  const unsigned nC = static_cast<unsigned>((n_keys + (1ull << lgC) - 1) >> lgC);
  const uintptr_t a = reinterpret_cast<uintptr_t>(mask);
  const int mbv = (mask_bytes == 1 && (a & 7u) == 0) ? 1 : (mask_bytes == 2 && (a & 15u) == 0) ? 2 : 0;
  static std::atomic<uint64_t> attr{0};  // dynamic LDS past 64 KiB: once per device (idempotent)
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (abytes > 64u * 1024u && dev >= 0 && dev < 64 && !((attr.load() >> dev) & 1u)) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&probe_munpermute_kernel<2048, 0>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&probe_munpermute_kernel<2048, 1>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&probe_munpermute_kernel<2048, 2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    attr.fetch_or(uint64_t(1) << dev);
  }
#define DLSM_MUNP(CC, MBV)                                                                                   \
  probe_munpermute_kernel<CC, MBV><<<nC, kBlock, abytes, s>>>(n_keys, groups, G, abytes, pos, answers, mask, \
                                                              mask_bytes)
#define DLSM_MUNP_C(CC)                  \
  do {                                   \
    if (mbv == 1) DLSM_MUNP(CC, 1);      \
    else if (mbv == 2) DLSM_MUNP(CC, 2); \
    else DLSM_MUNP(CC, 0);               \
  } while (0)
  if (lgC == 12) {
    if (abytes > 64u * 1024u) return hipErrorInvalidValue;
    DLSM_MUNP_C(4096);
  } else {
    DLSM_MUNP_C(2048);
  }
#undef DLSM_MUNP_C
#undef DLSM_MUNP
  return hipGetLastError();
}

hipError_t launch_version_route(const VersionDev& v, KeyDesc keys, uint64_t snapshot, uint64_t* slot_mask,
                                uint32_t* level_file, uint32_t* hv, uint32_t* gl, hipStream_t s) {
  if (keys.n == 0) return hipSuccess;
  const bool k20 = keys.offsets == nullptr && keys.key_len == 20 && keys.suffix == 0 &&
                   (reinterpret_cast<uintptr_t>(keys.bytes) & 3u) == 0;
  const bool route = hv != nullptr;
  uint32_t nf = v.n_l0;
  for (int lv = 1; lv < kNumLevels; lv++) nf = std::max(nf, v.lvl_begin[lv] + v.lvl_count[lv]);
  // $DLSM_VERSION_LDS (A/B): 0 the lane-per-lookup kernel; 2 / 3 / 4 / 5 the
  // wave-queued kernel with GT >= 1 / 2 / 3 / 4 even when more tables fit
  static const int lds_mode = [] {
    const char* e = getenv("DLSM_VERSION_LDS");
    return e ? atoi(e) : 1;
  }();
  // the LDS this device gives one workgroup (at most the kernel's 160 KiB)
  int dev = 0;
  (void)hipGetDevice(&dev);
  const size_t lds_cap = std::min(kVLdsMax, device_lds_max(dev));
  int gt = lds_mode >= 2 ? std::min(lds_mode, 5) - 1 : 0;
  while (gt < 4 && version_lds_bytes(v.n_bnd, nf, gt) > lds_cap) gt++;
  const size_t lds = version_lds_bytes(v.n_bnd, nf, gt);
  // a queued probe task names its file in 16 bits: larger versions take the
  // lane-per-lookup kernel (as does a device whose LDS cannot hold even the
  // wave queues)
  if (lds_mode != 0 && lds <= lds_cap && nf <= 0xffffu && dev >= 0 && dev < 64) {
    // all files probed directly or through the queue share one probe count
    // in the common case (one bits_per_key): k = 6 unrolled
    const uint32_t g = static_cast<uint32_t>(std::min<uint64_t>((keys.n + kVRouteNT - 1) / kVRouteNT,
                                                                static_cast<uint64_t>(device_cus())));
#define DLSM_VLDS_GT(MM, RR, KK, GG)                                                                            \
  do {                                                                                                          \
    /* the dynamic-LDS ceiling, once per device (builder threads race here: */                                 \
    /* the attribute call is idempotent, the flag word atomic) */                                               \
    static std::atomic<uint64_t> attr{0};                                                                       \
    if (!((attr.load(std::memory_order_acquire) >> dev) & 1u)) {                                                \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&version_lds_kernel<MM, RR, KK, GG>),             \
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds_cap));        \
      attr.fetch_or(uint64_t(1) << dev, std::memory_order_acq_rel);                                             \
    }                                                                                                           \
    version_lds_kernel<MM, RR, KK, GG><<<g, kVRouteNT, lds, s>>>(v, keys, snapshot, slot_mask, level_file, hv, gl, \
                                                                 nf);                                           \
  } while (0)
#define DLSM_VLDS(MM, RR, KK)                 \
  do {                                        \
    if (gt == 0)                              \
      DLSM_VLDS_GT(MM, RR, KK, 0);            \
    else if (gt == 1)                         \
      DLSM_VLDS_GT(MM, RR, KK, 1);            \
    else if (gt == 2)                         \
      DLSM_VLDS_GT(MM, RR, KK, 2);            \
    else if (gt == 3)                         \
      DLSM_VLDS_GT(MM, RR, KK, 3);            \
    else                                      \
      DLSM_VLDS_GT(MM, RR, KK, 4);            \
  } while (0)
    if (v.k_all == 6) {
      if (k20 && route) DLSM_VLDS(KM_K20, true, 6);
      else if (k20) DLSM_VLDS(KM_K20, false, 6);
      else if (route) DLSM_VLDS(KM_GENERIC, true, 6);
      else DLSM_VLDS(KM_GENERIC, false, 6);
    } else {
      if (k20 && route) DLSM_VLDS(KM_K20, true, 0);
      else if (k20) DLSM_VLDS(KM_K20, false, 0);
      else if (route) DLSM_VLDS(KM_GENERIC, true, 0);
      else DLSM_VLDS(KM_GENERIC, false, 0);
    }
#undef DLSM_VLDS
#undef DLSM_VLDS_GT
    return hipGetLastError();
  }
  const unsigned g = static_cast<unsigned>((keys.n + kBlock - 1) / kBlock);
  if (k20 && route)
    version_probe_kernel<KM_K20, true><<<g, kBlock, 0, s>>>(v, keys, snapshot, slot_mask, level_file, hv, gl);
  else if (k20)
    version_probe_kernel<KM_K20, false><<<g, kBlock, 0, s>>>(v, keys, snapshot, slot_mask, level_file);
  else if (route)
    version_probe_kernel<KM_GENERIC, true><<<g, kBlock, 0, s>>>(v, keys, snapshot, slot_mask, level_file, hv, gl);
  else
    version_probe_kernel<KM_GENERIC, false><<<g, kBlock, 0, s>>>(v, keys, snapshot, slot_mask, level_file);
  return hipGetLastError();
}

hipError_t launch_version_probe(const VersionDev& v, KeyDesc keys, uint64_t snapshot,
                                uint64_t* slot_mask, uint32_t* level_file, hipStream_t s) {
  return launch_version_route(v, keys, snapshot, slot_mask, level_file, nullptr, nullptr, s);
}

constexpr int kVPartNT = 1024;

hipError_t launch_version_partition(const uint32_t* hv, const uint32_t* gl, uint64_t n, uint32_t g0, uint32_t S,
                                    uint32_t* entries, uint16_t* pos, uint16_t* tab, uint32_t* gcnt,
                                    uint32_t* plan, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (S < 1 || S > kVMaxSlices) return hipErrorInvalidValue;
  const unsigned nC = static_cast<unsigned>((n + kVChunk - 1) / kVChunk);
  version_partition_kernel<kVPartNT><<<nC, kVPartNT, 0, s>>>(hv, gl, n, g0, S, entries, pos, tab, gcnt);
  version_plan_kernel<<<1, 1024, 0, s>>>(gcnt, S, kVPlanBudget, plan);
  return hipGetLastError();
}

hipError_t launch_version_slices(const uint8_t* image, uint32_t L, int k, uint32_t S, uint32_t n_chunks,
                                 const uint32_t* entries, const uint16_t* tab, uint8_t* smask,
                                 const uint32_t* plan, hipStream_t s) {
  if (n_chunks == 0) return hipSuccess;
  if (S < 1 || S > kVMaxSlices || L == 0) return hipErrorInvalidValue;
  constexpr int NT = DLSM_PROBE_NT;
  constexpr uint32_t R = 1u << kVSliceLg;
  const uint32_t grid = S + kVPlanBudget;  // >= the plan's parts: sum max(1, ceil(u / target)) <= S + budget
  // packed image of one member (LGW 0): the filters' own line bytes, answer in bit 0
  if (k == 6)
    probe_slice_kernel<kVSliceLg, 0, 6, NT, kVChunk, kVRegion><<<grid, NT, 0, s>>>(
        image, L, R, 0u, k, S, n_chunks, entries, tab, smask, 1, plan);
  else
    probe_slice_kernel<kVSliceLg, 0, 0, NT, kVChunk, kVRegion><<<grid, NT, 0, s>>>(
        image, L, R, 0u, k, S, n_chunks, entries, tab, smask, 1, plan);
  return hipGetLastError();
}

hipError_t launch_version_unpermute(uint64_t n, const uint16_t* pos, const uint8_t* smask, uint8_t* abyte,
                                    uint64_t* slot_mask, int jbit, int n_sliced, uint64_t slots, bool first,
                                    bool last, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const unsigned nC = static_cast<unsigned>((n + kVChunk - 1) / kVChunk);
  version_unpermute_kernel<<<nC, kBlock, 0, s>>>(n, pos, smask, abyte, slot_mask, jbit, n_sliced, slots,
                                                 first ? 1 : 0, last ? 1 : 0);
  return hipGetLastError();
}

// FilterBlockReader::KeyMayMatch(block_offset, key), table/filter_block.cc:
// 117-142, over one filter block (device), one thread per key.
template <int MODE>
__global__ __launch_bounds__(kBlock) void filter_block_probe_kernel(const uint8_t* __restrict__ blk,
                                                                    uint64_t n, KeyDesc kd,
                                                                    const uint64_t* __restrict__ offs,
                                                                    uint8_t* __restrict__ out) {
  const uint64_t i = blockIdx.x * static_cast<uint64_t>(kBlock) + threadIdx.x;
  if (i >= kd.n) return;
  uint8_t r = 1;  // "Errors are treated as potential matches"
  if (n >= 5) {
    const uint32_t base_lg = blk[n - 1] & 63u;  // size_t(char) >> on x86: count mod 64
    const uint32_t last_word = dec32_dev(blk + n - 5);
    if (last_word <= n - 5) {
      const uint64_t num = (n - 5 - last_word) / 4;
      const uint64_t index = offs[i] >> base_lg;
      if (index < num) {
        const uint8_t* o = blk + last_word + index * 4;
        const uint32_t start = dec32_dev(o), limit = dec32_dev(o + 4);
        if (start <= limit && limit <= last_word) {
          // BloomFilterPolicy::KeyMayMatch(key, filter), util/bloom.cc:57-81
          const uint64_t len = limit - start;
          const uint8_t* f = blk + start;
          if (len < 2) {
            r = 0;
          } else {
            const int k = static_cast<int>(static_cast<int8_t>(f[len - 1]));
            if (k > 0 && k <= 30) {
              const uint64_t bits = (len - 1) * 8;
              uint32_t h = key_hash<MODE>(kd, i);
              const uint32_t delta = bloom_delta(h);
              for (int q = 0; q < k; q++) {
                const uint32_t bp = bits > 0xffffffffull ? h : h % static_cast<uint32_t>(bits);
                if (((f[bp >> 3] >> (bp & 7u)) & 1u) == 0) {
                  r = 0;
                  break;
                }
                h += delta;
              }
            }
          }
        } else if (start == limit) {
          r = 0;  // empty filters do not match any keys
        }
      }
    }
  }
  out[i] = r;
}

hipError_t launch_filter_block_probe(const uint8_t* blk, uint64_t len, KeyDesc keys,
                                     const uint64_t* block_offsets, uint8_t* out, hipStream_t s) {
  if (keys.n == 0) return hipSuccess;
  const unsigned g = static_cast<unsigned>((keys.n + kBlock - 1) / kBlock);
  if (keys.offsets == nullptr && keys.key_len == 20 && keys.suffix == 0 &&
      (reinterpret_cast<uintptr_t>(keys.bytes) & 3u) == 0)
    filter_block_probe_kernel<KM_K20><<<g, kBlock, 0, s>>>(blk, len, keys, block_offsets, out);
  else
    filter_block_probe_kernel<KM_GENERIC><<<g, kBlock, 0, s>>>(blk, len, keys, block_offsets, out);
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

hipError_t launch_legacy_partition(const LegacyTileJobDev* jobs, const uint32_t* chunk0s, int n_jobs,
                                   uint32_t total_chunks, uint16_t* entries, uint16_t* tab, int variant,
                                   int mode, hipStream_t s) {
  if (total_chunks == 0) return hipSuccess;
#define DLSM_LPART(MM, KM, ST, TM) \
  legacy_partition_kernel<MM, KM, ST, TM><<<total_chunks, kLegacyPartBlock, 0, s>>>(jobs, chunk0s, n_jobs, entries, tab)
#define DLSM_LPART_V(MM)                                                   \
  do {                                                                     \
    if (variant == 0) DLSM_LPART(MM, kLegacyKmaxA, kLegacyStageA, kLegacyTilesA); \
    else DLSM_LPART(MM, kLegacyKmaxB, kLegacyStageB, kLegacyTilesB);          \
  } while (0)
  if (mode == KM_K20) DLSM_LPART_V(KM_K20);
  else if (mode == KM_K28) DLSM_LPART_V(KM_K28);
  else DLSM_LPART_V(KM_GENERIC);
#undef DLSM_LPART_V
#undef DLSM_LPART
  return hipGetLastError();
}

hipError_t launch_legacy_slices(const LegacyTileJobDev* jobs, const uint32_t* slice0s, int n_jobs,
                                uint32_t total_slices, const uint16_t* entries, const uint16_t* tab, int tps_lg,
                                hipStream_t s) {
  if (total_slices == 0) return hipSuccess;
  switch (tps_lg) {
#define DLSM_LSL(T) \
  case T: legacy_slice_kernel<T><<<total_slices, kLegacySliceBlock, 0, s>>>(jobs, slice0s, n_jobs, entries, tab); break
    DLSM_LSL(0);
    DLSM_LSL(1);
    DLSM_LSL(2);
    DLSM_LSL(3);
    DLSM_LSL(4);
#undef DLSM_LSL
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dlsm
