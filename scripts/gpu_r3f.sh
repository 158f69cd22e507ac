#!/usr/bin/env bash
# Round-3 session F: A/B of two window sets in flight (walk depth 2) for the
# probe (pd2) and build (bd2) slice passes at the full job and at the N = 4 /
# N = 8 shares, plus the non-temporal probe loads (ntl0 = plain), interleaved.
set -o pipefail
OUT=${1:-gpurun_out/r3f}
mkdir -p "$OUT"
export TMPDIR=/tmp
for SHARE in "--tables 16 --lookups 100000000" "--tables 2 --lookups 12500000" "--tables 4 --lookups 25000000"; do
  tag=$(echo $SHARE | awk '{print "t"$2}')
  for r in 1 2 3; do
    for v in base pd2 bd2 pd2bd2 ntl0; do
      if [ $v = base ]; then envs="DLSM_X=0"; else envs="DLSM_LIB_VARIANT=$v"; fi
      env $envs timeout -k 10 120 python bench.py --native --steps 100 --warmup 10 $SHARE \
        > "$OUT/${tag}_${v}_r$r.json" 2> "$OUT/${tag}_${v}_r$r.err" || exit 5
    done
  done
done
g++ -std=c++17 -O2 -fno-rtti -fno-exceptions -pthread -I include tests/cpp/concurrent_builders.cc \
  -L dlsm_amd/lib -ldlsm_bloom -L oracle -loracle -Wl,-rpath,$PWD/dlsm_amd/lib -Wl,-rpath,$PWD/oracle \
  -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -o "$OUT/cb" || exit 3
for r in 1 2; do
  for mode in hash ctx; do
    for t in 1 4 8 16; do
      timeout -k 10 200 "$OUT/cb" $t 8 153846 $mode >> "$OUT/concurrent_builders.jsonl" 2>> "$OUT/cb.err" || exit 4
    done
  done
done
