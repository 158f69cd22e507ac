#!/usr/bin/env bash
# Round-3 session Q: probe shape knobs at the N = 8 / N = 4 shares with the
# pass events sampled (native runner, 100 steps, 3 interleaved rounds):
# 64 KiB probe slices (--probe-slice-lg 7, two workgroups per CU) and
# 16,384-key probe chunks, against the defaults; overlap off for reference.
set -o pipefail
OUT=${1:-gpurun_out/r3q}
mkdir -p "$OUT"
for r in 1 2 3; do
  for share in "2 12500000" "4 25000000"; do
    set -- $share
    for spec in "base:" "slg7:--probe-slice-lg 7" "clg14:--probe-chunk-lg 14" "noover:--overlap off"; do
      label=${spec%%:*}; extra=${spec#*:}
      timeout -k 10 200 python3 bench.py --native --tables $1 --lookups $2 --steps 100 --warmup 10 --no-cpu --no-e2e $extra \
        > "$OUT/t$1_${label}_$r.json" 2> "$OUT/t$1_${label}_$r.err" || exit 2
      echo "t$1 $label r$r $(python3 -c "import json; d=json.loads(open('$OUT/t$1_${label}_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'build', d['build']['ms'], 'probe', d['probe']['ms'])")" >> "$OUT/summary.txt"
    done
  done
done
