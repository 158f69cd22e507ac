// Diagnostic (timing only, run by hand on a GPU box; results under profiles/):
// where the legacy-format partition pass (legacy_partition_kernel) spends its
// time.  The product kernels are included as they are; the ablations below
// are copies of the partition with phases removed -- their outputs are wrong
// by design and nothing reads them.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tests/diag/legacy_part_abl.hip -o /tmp/lpa && /tmp/lpa
#include "../../dlsm_amd/csrc/bloom_kernels.hip"

#include <cstdio>
#include <vector>

namespace dlsm {
namespace {

// V: 0 full (as the product), 1 no count pass (scatter with a fixed bucket
// capacity), 2 no scatter (count + scan + table + store), 3 no LDS atomics
// (hash + positions + store), 4 hash only (loads + hash, one store per thread)
template <int V>
__global__ __launch_bounds__(kLegacyPartBlock) void abl_kernel(const LegacyTileJobDev* __restrict__ jobs,
                                                              const uint32_t* __restrict__ chunk0s, int n_jobs,
                                                              uint16_t* __restrict__ entries, uint16_t* __restrict__ tab) {
  constexpr int NT = kLegacyPartBlock;
  constexpr int C = kLegacyChunk;
  constexpr int PER = C / NT;
  constexpr int KMAX = kLegacyKmaxA;
  constexpr uint32_t STAGE = kLegacyStageA, TMAX = kLegacyTilesA;
  constexpr int TKV = K20Tile<NT, tile_kpt<20>(), 20>::kVec;
  constexpr int SV = static_cast<int>(STAGE / 8u);
  constexpr int TVB = TKV > SV ? TKV : SV;
  __shared__ __attribute__((aligned(16))) uint4 tile[TVB];
  __shared__ uint32_t hist[TMAX + 1];
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
  hash_chunk<KM_K20, NT, PER>(J.keys, first, nk, tile, h);
  uint16_t* out = entries + J.entry0 + static_cast<uint64_t>(c) * J.region;
  if constexpr (V == 4) {
    uint32_t x = 0;
#pragma unroll
    for (int r = 0; r < PER; r++) x ^= h[r];
    out[tid] = static_cast<uint16_t>(x);
    return;
  }
  const uint32_t nT = J.n_tiles, bits = J.bits, magic = J.magic;
  const int k = J.k;
  uint16_t* stage = reinterpret_cast<uint16_t*>(tile);
  if constexpr (V == 3) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < PER; r++) {
      uint32_t hh = h[r];
      const uint32_t delta = bloom_delta(hh);
#pragma unroll
      for (int q = 0; q < KMAX; q++) {
        if (q < k) stage[(r * KMAX + q) * NT + tid] = static_cast<uint16_t>(fastmod(hh, bits, magic));
        hh += delta;
      }
    }
    __syncthreads();
    store_chunk_u16<NT>(out, stage, static_cast<uint32_t>(k) * C);
    return;
  }
  for (uint32_t b = tid; b <= nT; b += NT) hist[b] = 0;
  __syncthreads();
  if constexpr (V != 1) {
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
    for (uint32_t b = tid; b < nT; b += NT) hist[b] += (0u - hist[b]) & 7u;
    __syncthreads();
  } else {
    const uint32_t cap = (static_cast<uint32_t>(k) * C / nT + 32u) & ~7u;
    for (uint32_t b = tid; b < nT; b += NT) hist[b] = cap;
    __syncthreads();
  }
  const uint32_t total = block_excl_scan_lds<NT>(hist, static_cast<int>(nT + 1), wsum);
  uint16_t* trow = tab + J.tab0 + static_cast<uint64_t>(c) * (nT + 1);
  for (uint32_t b = tid; b <= nT; b += NT) trow[b] = static_cast<uint16_t>(hist[b]);
  __syncthreads();
  if constexpr (V != 2) {
#pragma unroll
    for (int r = 0; r < PER; r++) {
      const bool live = static_cast<uint32_t>(r * NT + tid) < nk;
      uint32_t hh = h[r];
      const uint32_t delta = bloom_delta(hh);
#pragma unroll
      for (int q = 0; q < KMAX; q++) {
        if (live && q < k) {
          const uint32_t bp = fastmod(hh, bits, magic);
          const uint32_t slot = atomicAdd(&hist[bp >> kLegacyTileLg], 1u);
          stage[min(slot, STAGE - 1u)] = static_cast<uint16_t>(bp);
        }
        hh += delta;
      }
    }
  }
  __syncthreads();
  store_chunk_u16<NT>(out, stage, min(total, STAGE));
}

__global__ void fill_keys(uint32_t* p, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) {
    uint32_t x = static_cast<uint32_t>(i) * 0x9E3779B9u;
    x ^= x >> 15;
    x *= 0x85EBCA6Bu;
    p[i] = x ^ (x >> 13);
  }
}

}  // namespace
}  // namespace dlsm

using namespace dlsm;

int main() {
  const int T = 16;
  const uint64_t N = 1600000;
  const int k = 6;
  uint8_t* keys = nullptr;
  (void)hipMalloc(&keys, T * N * 20 + 64);
  fill_keys<<<4096, 256>>>(reinterpret_cast<uint32_t*>(keys), T * N * 5);
  std::vector<LegacyTileJobDev> hj(T);
  std::vector<uint32_t> starts(T);
  uint64_t entry = 0, tabw = 0;
  uint32_t chunk = 0;
  const uint32_t bits = static_cast<uint32_t>(N * 10);
  const uint32_t nT = (bits + 65535) >> 16;
  for (int j = 0; j < T; j++) {
    LegacyTileJobDev& d = hj[j];
    d.keys = KeyDesc{keys + j * N * 20, nullptr, N, 20, 0};
    d.bits = bits;
    d.magic = fastmod_magic(bits);
    d.n_tiles = nT;
    d.region = legacy_region(k, nT);
    d.n_chunks = static_cast<uint32_t>((N + kLegacyChunk - 1) / kLegacyChunk);
    d.chunk0 = chunk;
    d.entry0 = entry;
    d.tab0 = tabw;
    d.k = k;
    starts[j] = chunk;
    entry += static_cast<uint64_t>(d.n_chunks) * d.region;
    tabw += static_cast<uint64_t>(d.n_chunks) * (nT + 1);
    chunk += d.n_chunks;
  }
  LegacyTileJobDev* dj = nullptr;
  uint32_t* ds = nullptr;
  uint16_t *ent = nullptr, *tab = nullptr;
  (void)hipMalloc(&dj, sizeof(LegacyTileJobDev) * T);
  (void)hipMalloc(&ds, sizeof(uint32_t) * T);
  (void)hipMalloc(&ent, entry * 2 + 64);
  (void)hipMalloc(&tab, tabw * 2 + 64);
  (void)hipMemcpy(dj, hj.data(), sizeof(LegacyTileJobDev) * T, hipMemcpyHostToDevice);
  (void)hipMemcpy(ds, starts.data(), sizeof(uint32_t) * T, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[5] = {"full", "no_count_pass", "no_scatter", "no_lds_atomics", "hash_only"};
  for (int round = 0; round < 2; round++) {
    for (int v = 0; v < 5; v++) {
      auto launch = [&] {
        switch (v) {
          case 0: abl_kernel<0><<<chunk, kLegacyPartBlock>>>(dj, ds, T, ent, tab); break;
          case 1: abl_kernel<1><<<chunk, kLegacyPartBlock>>>(dj, ds, T, ent, tab); break;
          case 2: abl_kernel<2><<<chunk, kLegacyPartBlock>>>(dj, ds, T, ent, tab); break;
          case 3: abl_kernel<3><<<chunk, kLegacyPartBlock>>>(dj, ds, T, ent, tab); break;
          default: abl_kernel<4><<<chunk, kLegacyPartBlock>>>(dj, ds, T, ent, tab); break;
        }
      };
      for (int w = 0; w < 3; w++) launch();
      (void)hipEventRecord(e0);
      const int R = 20;
      for (int r = 0; r < R; r++) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      std::printf("{\"variant\": \"%s\", \"chunk\": %d, \"threads\": %d, \"us\": %.1f}\n", names[v], kLegacyChunk,
                  kLegacyPartBlock, ms * 1000.0 / R);
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
