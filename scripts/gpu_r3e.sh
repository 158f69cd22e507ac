#!/usr/bin/env bash
# Round-3 session E: the default bench line (N = 1 now timed by the native
# runner) and the Python-loop form; knob sweep at the N = 8 / N = 4 shares;
# concurrent builders with block-hashed AddKey.
set -o pipefail
OUT=${1:-gpurun_out/r3e}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 2
timeout -k 10 200 python bench.py --python-loop --no-cpu --no-e2e > "$OUT/bench_pyloop.json" 2> "$OUT/bench_pyloop.err" || exit 2
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --no-e2e > "$OUT/ntl1_r$r.json" 2> "$OUT/ntl1_r$r.err" || exit 2
  DLSM_LIB_VARIANT=ntl0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --no-e2e \
    > "$OUT/ntl0_r$r.json" 2> "$OUT/ntl0_r$r.err" || exit 2
done
run() {  # name "ENV=.." extra-bench-args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 120 python bench.py --native --steps 100 --warmup 10 $SHARE "$@" \
    > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 5
}
for SHARE in "--tables 2 --lookups 12500000" "--tables 4 --lookups 25000000"; do
  tag=$(echo $SHARE | awk '{print "t"$2}')
  for r in 1 2; do
    run ${tag}_base_r$r "DLSM_X=0"
    run ${tag}_grid0_r$r "DLSM_PART_GRID_PER_CU=0"
    run ${tag}_grid3_r$r "DLSM_PART_GRID_PER_CU=3"
    run ${tag}_noover_r$r "DLSM_X=0" --overlap off
    run ${tag}_chunk12_r$r "DLSM_X=0" --probe-chunk-lg 12
  done
done
g++ -std=c++17 -O2 -fno-rtti -fno-exceptions -pthread -I include tests/cpp/concurrent_builders.cc \
  -L dlsm_amd/lib -ldlsm_bloom -L oracle -loracle -Wl,-rpath,$PWD/dlsm_amd/lib -Wl,-rpath,$PWD/oracle \
  -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -o "$OUT/cb" || exit 3
for mode in hash ctx; do
  for t in 1 4 8 16; do
    timeout -k 10 200 "$OUT/cb" $t 8 153846 $mode >> "$OUT/concurrent_builders.jsonl" 2>> "$OUT/cb.err" || exit 4
  done
done
