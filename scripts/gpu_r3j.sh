#!/usr/bin/env bash
# Round-3 session J: host-API builds store filters and lengths straight to
# page-locked host memory (one synchronisation, no D2H commands) and the
# adapter streams AddKey's hashes to the device while AddKey runs
# (dlsm_stage_hashes).  Parity tests of every host-API user, then concurrent
# builders: hash (streamed) vs hash-finish (all hashes in Finish) vs ctx, and
# a kernel/copy trace of one thread.
set -o pipefail
OUT=${1:-gpurun_out/r3j}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_hashed_build.py tests/test_gpu_adapter.py tests/test_gpu_parity.py tests/test_internal_keys.py \
  tests/test_filter_block.py tests/test_gpu_workspace.py > "$OUT/pytest.log" 2>&1 || exit 2
g++ -std=c++17 -O2 -fno-rtti -fno-exceptions -pthread -I include tests/cpp/concurrent_builders.cc \
  -L dlsm_amd/lib -ldlsm_bloom -L oracle -loracle -Wl,-rpath,$PWD/dlsm_amd/lib -Wl,-rpath,$PWD/oracle \
  -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -o "$OUT/cb" || exit 3
for r in 1 2 3; do
  for mode in hash hash-finish ctx; do
    for t in 1 4 8 16; do
      timeout -k 10 120 "$OUT/cb" $t 8 153846 $mode >> "$OUT/concurrent_builders.jsonl" 2>> "$OUT/cb.err" || exit 4
    done
  done
done
for mode in hash hash-finish; do
  timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d "$OUT/prof_$mode" -o run -- "$OUT/cb" 1 8 153846 $mode > "$OUT/prof_$mode.jsonl" 2> "$OUT/prof_$mode.err" || exit 5
done
