#!/usr/bin/env bash
# Round-3 session H: the one-launch build of small hashed jobs
# (full_small_hashed_kernel): its parity tests, then concurrent builder
# threads hashing in AddKey with it on (DLSM_SMALL_BUILD=1) and off (count +
# partition + slice), interleaved, plus 16 threads with 16 hardware queues.
set -o pipefail
OUT=${1:-gpurun_out/r3h}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_hashed_build.py tests/test_gpu_adapter.py > "$OUT/pytest.log" 2>&1 || exit 2
g++ -std=c++17 -O2 -fno-rtti -fno-exceptions -pthread -I include tests/cpp/concurrent_builders.cc \
  -L dlsm_amd/lib -ldlsm_bloom -L oracle -loracle -Wl,-rpath,$PWD/dlsm_amd/lib -Wl,-rpath,$PWD/oracle \
  -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -o "$OUT/cb" || exit 3
for r in 1 2 3; do
  for small in 1 0; do
    for t in 1 4 8 16; do
      DLSM_SMALL_BUILD=$small timeout -k 10 120 "$OUT/cb" $t 8 153846 hash \
        | sed "s/^{/{\"small\": $small, /" >> "$OUT/concurrent_builders.jsonl" 2>> "$OUT/cb.err" || exit 4
    done
  done
  for small in 1 0; do
    GPU_MAX_HW_QUEUES=16 DLSM_SMALL_BUILD=$small timeout -k 10 120 "$OUT/cb" 16 8 153846 hash \
      | sed "s/^{/{\"small\": $small, \"hwq\": 16, /" >> "$OUT/concurrent_builders.jsonl" 2>> "$OUT/cb.err" || exit 4
  done
done
