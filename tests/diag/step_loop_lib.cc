// Diagnostic: the bench step loop in C, called ONCE from a Python process
// that has torch loaded (tests/diag/run_step_loop_lib.py): K x (batched
// build + probe) through the C ABI with no Python between the calls.  Tells
// whether bench.py's ~10 us call-boundary gaps come from the per-call
// Python/ctypes path or from the torch process's runtime state.
#include <cstdint>

#include "dlsm_bloom.h"

extern "C" int step_loop_run(dlsm_ctx* bctx, const dlsm_build_job* jobs, int n_jobs, int bpk,
                             uint64_t* lens_dev, dlsm_ctx* pctx, const dlsm_filterset* fs,
                             const dlsm_keyset* keys, uint8_t* mask_dev, int steps) {
  for (int i = 0; i < steps; i++) {
    int s = dlsm_bloom_full_build_dev(bctx, jobs, n_jobs, bpk, lens_dev);
    if (s) return s;
    s = dlsm_bloom_full_probe_dev(pctx, fs, keys, mask_dev);
    if (s) return s;
  }
  return 0;
}
