#!/usr/bin/env bash
# Round-3 session L: AddKey's 20-byte fast path (two fixed-size copies, no
# length record) vs the previous adapter (tests/diag/ab_old_adapter, the
# committed header), interleaved: concurrent builders in hash mode.
set -o pipefail
OUT=${1:-gpurun_out/r3l}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in new old; do
  inc=include; [ $v = old ] && inc=tests/diag/ab_old_adapter
  g++ -std=c++17 -O2 -fno-rtti -fno-exceptions -pthread -I $inc tests/cpp/concurrent_builders.cc \
    -L dlsm_amd/lib -ldlsm_bloom -L oracle -loracle -Wl,-rpath,$PWD/dlsm_amd/lib -Wl,-rpath,$PWD/oracle \
    -Wl,-rpath,/opt/rocm/lib -L/opt/rocm/lib -o "$OUT/cb_$v" || exit 3
done
timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_gpu_adapter.py \
  > "$OUT/pytest.log" 2>&1 || exit 2
for r in 1 2 3 4; do
  for v in new old; do
    for t in 1 16; do
      timeout -k 10 120 "$OUT/cb_$v" $t 8 153846 hash | sed "s/^{/{\"adapter\": \"$v\", /" \
        >> "$OUT/concurrent_builders.jsonl" 2>> "$OUT/cb.err" || exit 4
    done
  done
done
