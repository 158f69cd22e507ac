#!/usr/bin/env bash
# Round-3 session R: build partition chunk size (DLSM_BUILD_CHUNK 2048 / 8192
# variants vs the default 4096) at the whole job and the N = 4 / N = 8 shares;
# native runner, 100 steps, 3 interleaved rounds.
set -o pipefail
OUT=${1:-gpurun_out/r3r}
mkdir -p "$OUT"
for r in 1 2 3; do
  for share in "16 100000000" "4 25000000" "2 12500000"; do
    set -- $share
    for v in base bc2048 bc8192; do
      if [ $v = base ]; then unset DLSM_LIB_VARIANT; else export DLSM_LIB_VARIANT=$v; fi
      timeout -k 10 200 python3 bench.py --native --tables $1 --lookups $2 --steps 100 --warmup 10 --no-cpu --no-e2e \
        > "$OUT/t$1_${v}_$r.json" 2> "$OUT/t$1_${v}_$r.err" || exit 2
      echo "t$1 $v r$r $(python3 -c "import json; d=json.loads(open('$OUT/t$1_${v}_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'build', d['build']['ms'], 'probe', d['probe']['ms'])")" >> "$OUT/summary.txt"
    done
  done
done
unset DLSM_LIB_VARIANT
# parity of the variants' builds against the oracle (the build tests only)
for v in bc2048 bc8192; do
  DLSM_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_fullsize.py -k build tests/test_gpu_parity.py > "$OUT/pytest_$v.log" 2>&1 || exit 3
done
