#!/usr/bin/env bash
# Compile the dLSM reference's Bloom hot-path sources IN PLACE (no copies) into
# oracle/_ref/libref.so -- TEST INFRASTRUCTURE ONLY, this container only.
# Output stays under oracle/_ref/ (git-ignored).  No-op when /root/reference is
# absent (the GPU box).  See oracle/ref_driver.cc for what is and isn't built.
set -euo pipefail
REF=${DLSM_REFERENCE:-/root/reference}
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="$HERE/_ref"
if [ ! -d "$REF/util" ]; then
  echo "build_ref: $REF not present; skipping reference oracle build"
  exit 0
fi
mkdir -p "$OUT"
g++ -std=c++17 -O2 -DNDEBUG -DHAVE_SNAPPY=0 -DTimberSaw_PLATFORM_POSIX=1 -fPIC -shared \
  -I"$REF" -I"$REF/include" \
  "$HERE/ref_driver.cc" "$REF/util/hash.cc" "$REF/util/bloom.cc" "$REF/util/filter_policy.cc" \
  "$REF/util/crc32c.cc" \
  -o "$OUT/libref.so"
echo "build_ref: built $OUT/libref.so"
