#!/usr/bin/env bash
# Interleaved A/B of library variants (make variant TAG=... VFLAGS=...) on the
# legacy-format batch build alone (scripts/bench_legacy.py), 3 rounds.
#   bash scripts/ab_legacy_variants.sh base tag1 tag2 ...
set -o pipefail
for r in 1 2 3; do
  for v in "$@"; do
    if [ "$v" = base ]; then unset DLSM_LIB_VARIANT; else export DLSM_LIB_VARIANT=$v; fi
    timeout -k 10 120 python scripts/bench_legacy.py || exit 3
  done
done
