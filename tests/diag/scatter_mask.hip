// Diagnostic only (VERDICT r2 "next" 2b): what the probe's slice pass would
// pay to write each key's final mask byte itself -- one byte store per key at
// the key's own position inside its 8,192-key chunk -- instead of writing the
// answers in bucket order (one dword per lane per 4 entries) and gathering
// them back to key order in a separate unpermute pass.
//
// Both kernels walk the same bucket-ordered entries the way the slice pass
// does: workgroup (slice s, part p) visits chunks c of its part in order and,
// per chunk, the run of entries bucketed to s; each lane takes 4 consecutive
// entries (one 16-byte unit).  Per entry the scattered kernel loads the key's
// in-chunk index (u16, bucket order) and stores the answer byte at
// mask[c * C + index]; the coalesced kernel stores the 4 answer bytes as one
// dword at the entries' own bucket positions (today's slice pass).  The
// answer value is a stand-in (entry index hash): the LDS probes are not
// modelled, only the stores and the index loads.
// tests/diag/run_scatter_mask.py builds the buckets and drives it.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
constexpr int kNT = 1024;

template <bool SCATTER>
__global__ __launch_bounds__(kNT) void walk_kernel(const uint32_t* __restrict__ run_off,  // [nC][S+1], in units
                                                   const uint16_t* __restrict__ idx,      // bucket order, [nC][CR]
                                                   uint8_t* __restrict__ out, uint32_t S, uint32_t nC,
                                                   uint32_t C, uint32_t CR, int parts) {
  const uint32_t s = blockIdx.x % S, p = blockIdx.x / S;
  const uint32_t c_lo = static_cast<uint32_t>(static_cast<uint64_t>(p) * nC / parts);
  const uint32_t c_hi = static_cast<uint32_t>(static_cast<uint64_t>(p + 1) * nC / parts);
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint32_t c = c_lo + wave; c < c_hi; c += kNT / 64) {
    const uint32_t* ro = run_off + static_cast<uint64_t>(c) * (S + 1);
    const uint32_t u0 = ro[s], u1 = ro[s + 1];  // the run's 16-byte units (4 entries each)
    for (uint32_t u = u0 + lane; u < u1; u += 64) {
      const uint64_t e = static_cast<uint64_t>(c) * CR + 4u * u;  // first entry of the unit
      const uint32_t a = static_cast<uint32_t>(e * 0x9e3779b9u);
      if constexpr (SCATTER) {
        const uint2 ix = *reinterpret_cast<const uint2*>(idx + e);  // 4 u16 indices
        uint8_t* m = out + static_cast<uint64_t>(c) * C;
        const uint32_t q[4] = {ix.x & 0xffffu, ix.x >> 16, ix.y & 0xffffu, ix.y >> 16};
#pragma unroll
        for (int j = 0; j < 4; j++)
          if (q[j] != 0xffffu) m[q[j]] = static_cast<uint8_t>(a >> (8 * j));  // 0xffff: bucket padding
      } else {
        reinterpret_cast<uint32_t*>(out)[e / 4] = a;
      }
    }
  }
}
}  // namespace

extern "C" int scatter_mask_launch(int scatter, const uint32_t* run_off, const uint16_t* idx, uint8_t* out,
                                   uint32_t S, uint32_t nC, uint32_t C, uint32_t CR, int parts) {
  const dim3 g(S * parts), b(kNT);
  if (scatter)
    walk_kernel<true><<<g, b>>>(run_off, idx, out, S, nC, C, CR, parts);
  else
    walk_kernel<false><<<g, b>>>(run_off, idx, out, S, nC, C, CR, parts);
  return static_cast<int>(hipGetLastError());
}
