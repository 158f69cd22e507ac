#!/usr/bin/env bash
# Round-3 session Z: the probe partition's position stores plain
# (Infinity-Cache-allocating; variant pp) instead of non-temporal, so the
# unpermute may re-read part of the 200 MB of positions from the cache; ntl0 =
# pp + plain entry/position loads.  Native runner, 100 steps, 3 interleaved
# rounds, whole job (default = build beside probe) and one stream; kernel
# stats of each.
set -o pipefail
OUT=${1:-gpurun_out/r3z}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2 3; do
  for ov in auto off; do
    for v in base pp ntl0; do
      if [ $v = base ]; then unset DLSM_LIB_VARIANT; else export DLSM_LIB_VARIANT=$v; fi
      timeout -k 10 200 python3 bench.py --native --overlap $ov --steps 100 --warmup 10 --no-cpu --no-e2e \
        > "$OUT/${ov}_${v}_$r.json" 2> "$OUT/${ov}_${v}_$r.err" || exit 3
      echo "$ov $v r$r $(python3 -c "import json; d=json.loads(open('$OUT/${ov}_${v}_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'build', d['build']['ms'], 'probe', d['probe']['ms'])")" >> "$OUT/summary.txt"
    done
  done
done
for v in base pp ntl0; do
  if [ $v = base ]; then unset DLSM_LIB_VARIANT; else export DLSM_LIB_VARIANT=$v; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$v" -o run -- \
    python3 bench.py --native --overlap off --steps 40 --warmup 5 --no-cpu --no-e2e > "$OUT/prof_$v.json" 2> "$OUT/prof_$v.err" || exit 4
done
