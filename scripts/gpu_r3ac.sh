#!/usr/bin/env bash
# Round-3 session AC: the build kernels' wave-ballot job lookup (new, default
# library) vs lane 0's binary search + barrier (variant "old") -- the change
# that was meant to be in session T's A/B but was left out of its library.
# Build parity tests first; native runner, 100 steps, 3 interleaved rounds.
set -o pipefail
OUT=${1:-gpurun_out/r3ac}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py tests/test_gpu_workspace.py tests/test_gpu_hashed_build.py tests/test_internal_keys.py \
  tests/test_gpu_adapter.py > "$OUT/pytest.log" 2>&1 || exit 2
for r in 1 2 3; do
  for share in "16 100000000" "2 12500000"; do
    set -- $share
    for v in old new; do
      if [ $v = old ]; then export DLSM_LIB_VARIANT=old; else unset DLSM_LIB_VARIANT; fi
      timeout -k 10 200 python3 bench.py --native --tables $1 --lookups $2 --steps 100 --warmup 10 --no-cpu --no-e2e \
        > "$OUT/t$1_${v}_$r.json" 2> "$OUT/t$1_${v}_$r.err" || exit 3
      echo "t$1 $v r$r $(python3 -c "import json; d=json.loads(open('$OUT/t$1_${v}_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'build', d['build']['ms'], 'probe', d['probe']['ms'])")" >> "$OUT/summary.txt"
    done
  done
done
