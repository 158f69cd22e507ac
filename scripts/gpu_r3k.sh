#!/usr/bin/env bash
# Round-3 session K: the whole GPU suite on the final host-API path (filters
# and lengths stored by the kernels into page-locked host memory), then
# concurrent builder threads (hash / ctx modes, 3 interleaved repetitions).
set -o pipefail
OUT=${1:-gpurun_out/r3k}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || exit 2
g++ -std=c++17 -O2 -fno-rtti -fno-exceptions -pthread -I include tests/cpp/concurrent_builders.cc \
  -L dlsm_amd/lib -ldlsm_bloom -L oracle -loracle -Wl,-rpath,$PWD/dlsm_amd/lib -Wl,-rpath,$PWD/oracle \
  -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -o "$OUT/cb" || exit 3
for r in 1 2 3; do
  for mode in hash ctx; do
    for t in 1 4 8 16; do
      timeout -k 10 120 "$OUT/cb" $t 8 153846 $mode >> "$OUT/concurrent_builders.jsonl" 2>> "$OUT/cb.err" || exit 4
    done
  done
done
