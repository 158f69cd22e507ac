#!/usr/bin/env bash
# Round-3 session T: the build kernels find their job with one wave-ballot
# over the jobs' first chunks / slices instead of a dependent binary search
# + the probe slice pass issues its first table-row loads before its image
# prologue + the unpermute loads its positions before staging the answers
# (new, default library) vs the previous library (variant "old");
# parity tests first; native runner, 100 steps, 3 interleaved rounds at the
# whole job and the N = 4 / N = 8 shares.
set -o pipefail
OUT=${1:-gpurun_out/r3t}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_walk_edges.py tests/test_gpu_packed_groups.py \
  tests/test_gpu_fullsize.py tests/test_gpu_workspace.py tests/test_gpu_hashed_build.py tests/test_internal_keys.py \
  > "$OUT/pytest.log" 2>&1 || exit 2
for r in 1 2 3; do
  for share in "2 12500000" "4 25000000" "16 100000000"; do
    set -- $share
    for v in old new; do
      if [ $v = old ]; then export DLSM_LIB_VARIANT=old; else unset DLSM_LIB_VARIANT; fi
      timeout -k 10 200 python3 bench.py --native --tables $1 --lookups $2 --steps 100 --warmup 10 --no-cpu --no-e2e \
        > "$OUT/t$1_${v}_$r.json" 2> "$OUT/t$1_${v}_$r.err" || exit 3
      echo "t$1 $v r$r $(python3 -c "import json; d=json.loads(open('$OUT/t$1_${v}_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'build', d['build']['ms'], 'probe', d['probe']['ms'])")" >> "$OUT/summary.txt"
    done
  done
done
unset DLSM_LIB_VARIANT
for t in "2 12500000" "16 100000000"; do
  set -- $t
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_t$1" -o run -- \
    python3 bench.py --native --tables $1 --lookups $2 --overlap off --steps 40 --warmup 5 --no-cpu --no-e2e \
    > "$OUT/prof_t$1.json" 2> "$OUT/prof_t$1.err" || exit 4
done
