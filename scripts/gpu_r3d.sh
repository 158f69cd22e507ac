#!/usr/bin/env bash
# Round-3 session D: host staging memory kinds; concurrent builders (ctx /
# hash, branch-free hash staging); the strong-scaling shares timed by the
# native runner (no profiler: per-step host cost is the C++ loop's).
set -o pipefail
OUT=${1:-gpurun_out/r3d}
mkdir -p "$OUT"
export TMPDIR=/tmp
/opt/rocm/bin/hipcc -O2 -std=c++17 --offload-arch=gfx950 tests/diag/host_staging.hip -o "$OUT/host_staging" || exit 3
timeout -k 10 120 "$OUT/host_staging" > "$OUT/host_staging.json" 2> "$OUT/host_staging.err" || exit 4
g++ -std=c++17 -O2 -fno-rtti -fno-exceptions -pthread -I include tests/cpp/concurrent_builders.cc \
  -L dlsm_amd/lib -ldlsm_bloom -L oracle -loracle -Wl,-rpath,$PWD/dlsm_amd/lib -Wl,-rpath,$PWD/oracle \
  -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -o "$OUT/cb" || exit 3
for mode in hash ctx; do
  for t in 1 4 8 16; do
    timeout -k 10 200 "$OUT/cb" $t 8 153846 $mode >> "$OUT/concurrent_builders.jsonl" 2>> "$OUT/cb.err" || exit 4
  done
done
for share in "16 100000000" "8 50000000" "4 25000000" "2 12500000"; do
  set -- $share
  timeout -k 10 300 python3 bench.py --native --tables $1 --lookups $2 --steps 100 --warmup 10 \
    > "$OUT/native_share_t$1.json" 2> "$OUT/native_share_t$1.err" || exit 6
done
timeout -k 10 300 python3 bench.py --gpus 8 --rehearse --steps 20 --warmup 5 > "$OUT/bench_g8r.json" 2> "$OUT/bench_g8r.err" || exit 7
