#!/usr/bin/env bash
# Round-3 session B: hashed-build + batcher parity, concurrent builder modes
# at 1/4/16 threads, and every streaming-kernel shape.  Each GPU step has its
# own limit; a test failure (rc 1) still lets the measurements run.
set -o pipefail
OUT=${1:-gpurun_out/r3b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hashed_build.py tests/test_gpu_adapter.py -m gpu -v \
  --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
g++ -std=c++17 -O2 -fno-rtti -fno-exceptions -pthread -I include tests/cpp/concurrent_builders.cc \
  -L dlsm_amd/lib -ldlsm_bloom -L oracle -loracle -Wl,-rpath,$PWD/dlsm_amd/lib -Wl,-rpath,$PWD/oracle \
  -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -o "$OUT/cb" || exit 3
for mode in ctx batch hash batch-hash; do
  for t in 1 4 16; do
    timeout -k 10 200 "$OUT/cb" $t 8 153846 $mode >> "$OUT/concurrent_builders.jsonl" 2>> "$OUT/cb.err" || exit 4
  done
done
timeout -k 10 300 python tests/diag/run_stream_variants.py > "$OUT/stream_variants.json" 2> "$OUT/stream_variants.err" &&
exit $rc
