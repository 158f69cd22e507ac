#!/usr/bin/env bash
# Round-3 session C: all GPU tests; balanced probe slices A/B (interleaved);
# concurrent builder modes at 1..16 threads; the strong-scaling shares
# (N = 2 / 4 / 8) under rocprofv3 --kernel-trace --stats.
set -o pipefail
OUT=${1:-gpurun_out/r3c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for bal in 1 0; do
    DLSM_PROBE_BALANCE=$bal timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu --no-e2e \
      > "$OUT/ab_bal${bal}_r$r.json" 2> "$OUT/ab_bal${bal}_r$r.err" || exit 5
  done
done
g++ -std=c++17 -O2 -fno-rtti -fno-exceptions -pthread -I include tests/cpp/concurrent_builders.cc \
  -L dlsm_amd/lib -ldlsm_bloom -L oracle -loracle -Wl,-rpath,$PWD/dlsm_amd/lib -Wl,-rpath,$PWD/oracle \
  -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -o "$OUT/cb" || exit 3
for mode in ctx hash batch batch-hash; do
  for t in 1 2 4 8 16; do
    timeout -k 10 200 "$OUT/cb" $t 8 153846 $mode >> "$OUT/concurrent_builders.jsonl" 2>> "$OUT/cb.err" || exit 4
  done
done
for w in 50 200; do
  timeout -k 10 200 "$OUT/cb" 16 8 153846 batch $w >> "$OUT/concurrent_builders.jsonl" 2>> "$OUT/cb.err" || exit 4
  timeout -k 10 200 "$OUT/cb" 16 8 153846 batch-hash $w >> "$OUT/concurrent_builders.jsonl" 2>> "$OUT/cb.err" || exit 4
done
for share in "8 50000000" "4 25000000" "2 12500000"; do
  set -- $share
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_t$1" -o run -- \
    python3 bench.py --tables $1 --lookups $2 --steps 50 --warmup 10 --no-cpu --no-e2e \
    > "$OUT/share_t$1.json" 2> "$OUT/share_t$1.err" || exit 6
done
exit $rc
