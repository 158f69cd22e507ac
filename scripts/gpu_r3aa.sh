#!/usr/bin/env bash
# Round-3 session AA: the persistent probe partition's grid under the
# overlapped step -- one workgroup per CU (leaving LDS for build partition
# workgroups beside it) vs the default two; native runner, 100 steps, 3
# interleaved rounds, whole job and N = 8 share.
set -o pipefail
OUT=${1:-gpurun_out/r3aa}
mkdir -p "$OUT"
for r in 1 2 3; do
  for share in "16 100000000" "2 12500000"; do
    set -- $share
    for g in 2 1; do
      DLSM_PART_GRID_PER_CU=$g timeout -k 10 200 python3 bench.py --native --tables $1 --lookups $2 --steps 100 \
        --warmup 10 --no-cpu --no-e2e > "$OUT/t$1_g${g}_$r.json" 2> "$OUT/t$1_g${g}_$r.err" || exit 3
      echo "t$1 grid$g r$r $(python3 -c "import json; d=json.loads(open('$OUT/t$1_g${g}_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'build', d['build']['ms'], 'probe', d['probe']['ms'])")" >> "$OUT/summary.txt"
    done
  done
done
