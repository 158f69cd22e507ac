#!/usr/bin/env bash
# Round-3 session I: where one builder thread's Finish spends its time --
# rocprofv3 kernel + memory-copy trace of concurrent_builders (1 and 16
# threads, hash mode) with the one-launch small build on and off.
set -o pipefail
OUT=${1:-gpurun_out/r3i}
mkdir -p "$OUT"
export TMPDIR=/tmp
g++ -std=c++17 -O2 -fno-rtti -fno-exceptions -pthread -I include tests/cpp/concurrent_builders.cc \
  -L dlsm_amd/lib -ldlsm_bloom -L oracle -loracle -Wl,-rpath,$PWD/dlsm_amd/lib -Wl,-rpath,$PWD/oracle \
  -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -o "$OUT/cb" || exit 3
for small in 0 1; do
  for t in 1 16; do
    DLSM_SMALL_BUILD=$small timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats \
      --output-format csv -d "$OUT/s${small}_t$t" -o run -- "$OUT/cb" $t 8 153846 hash \
      > "$OUT/s${small}_t$t.jsonl" 2> "$OUT/s${small}_t$t.err" || exit 4
  done
done
