// Diagnostic only: the minimal form of the commit-1c7c4c6 failure.  Every
// lane keeps a value loaded from memory (unique per lane and workgroup) live
// across an inline-asm statement that clobbers all 64 VGPRs, so the compiler
// must spill it to scratch and reload it; each lane counts reloads that came
// back different.  Built for 1,024-thread workgroups at 8 waves per SIMD
// (__launch_bounds__(1024, 8)), with 64 KiB of LDS (two workgroups per CU)
// or 88 KiB (one per CU).  tests/diag/run_spill_probe.py drives it.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {
constexpr int LDSKB = 64;

__global__ __launch_bounds__(1024, 8) void spill_probe_kernel(const uint32_t* __restrict__ in,
                                                              uint32_t* __restrict__ bad, int iters) {
  __shared__ uint32_t lds[LDSKB * 256];
  const uint32_t gid = blockIdx.x * 1024u + threadIdx.x;
  for (uint32_t i = threadIdx.x; i < LDSKB * 256u; i += 1024u) lds[i] = i ^ gid;
  __syncthreads();
  const uint32_t v = in[gid];
  uint32_t acc = lds[(threadIdx.x * 7u) % (LDSKB * 256u)];
  uint32_t nbad = 0;
  for (int it = 0; it < iters; it++) {
    asm volatile("s_nop 0" ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63");
    const uint32_t w = in[gid];  // the value the spilled copy must equal
    nbad += (v != w) ? 1u : 0u;
    acc += lds[(acc + it) % (LDSKB * 256u)];
  }
  bad[gid] = nbad + (acc == 0x9e3779b9u ? 1u << 31 : 0u);  // acc keeps the LDS reads alive
}

// The pre-fix kernel's own pattern: a wave prefix scan through __shfl_up
// (ds_bpermute) whose lane addresses are spilled across the clobber and
// reloaded for every scan, next to a sweep of the 64 KiB LDS array.
__device__ __forceinline__ uint32_t scan_shfl(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

__global__ __launch_bounds__(1024, 8) void spill_scan_kernel(const uint32_t* __restrict__ in,
                                                            uint32_t* __restrict__ bad, int iters) {
  __shared__ uint32_t lds[LDSKB * 256];
  const uint32_t gid = blockIdx.x * 1024u + threadIdx.x;
  for (uint32_t i = threadIdx.x; i < LDSKB * 256u; i += 1024u) lds[i] = i ^ gid;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  uint32_t acc = 0, nbad = 0;
  for (int it = 0; it < iters; it++) {
    asm volatile("s_nop 0" ::: "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15","v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31","v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55","v56","v57","v58","v59","v60","v61","v62","v63");
    const uint32_t x = in[gid] + static_cast<uint32_t>(it);
    const uint32_t s = scan_shfl(x & 0xffu);
    // expected: sum of (in[lane'] + it) & 0xff over lanes <= lane of this wave
    uint32_t want = 0;
    const uint32_t base = gid - lane;
    for (uint32_t l = 0; l <= lane; l++) want += (in[base + l] + static_cast<uint32_t>(it)) & 0xffu;
    nbad += (s != want) ? 1u : 0u;
    acc += lds[(acc + x) % (LDSKB * 256u)];
  }
  bad[gid] = nbad + (acc == 0x9e3779b9u ? 1u << 31 : 0u);
}
}  // namespace

// extra_lds_kb 0: two 1,024-thread workgroups per CU; 24: one.  kind 0: the
// spilled-value check; 1: the spilled-address scan.
extern "C" int spill_probe_launch(const uint32_t* in, uint32_t* bad, int blocks, int iters, int extra_lds_kb,
                                  int kind) {
  const size_t dyn = static_cast<size_t>(extra_lds_kb) * 1024;
  if (kind == 0)
    hipLaunchKernelGGL(spill_probe_kernel, dim3(blocks), dim3(1024), dyn, 0, in, bad, iters);
  else
    hipLaunchKernelGGL(spill_scan_kernel, dim3(blocks), dim3(1024), dyn, 0, in, bad, iters);
  if (hipGetLastError() != hipSuccess) return -1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
