#!/usr/bin/env bash
# Round-3 end: each GPU's share of the strong-scaling job on the final tree
# (native runner, build beside probe, pass events on 4 sampled steps), 100
# steps, 3 interleaved rounds on one box; and --gpus 2 / 4 rehearsed.
set -o pipefail
OUT=${1:-gpurun_out/r3ab}
mkdir -p "$OUT"
for r in 1 2 3; do
  for share in "16 100000000" "8 50000000" "4 25000000" "2 12500000"; do
    set -- $share
    timeout -k 10 200 python3 bench.py --native --tables $1 --lookups $2 --steps 100 --warmup 10 --no-cpu --no-e2e \
      > "$OUT/t$1_$r.json" 2> "$OUT/t$1_$r.err" || exit 3
    echo "t$1 r$r $(python3 -c "import json; d=json.loads(open('$OUT/t$1_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'value', d['value'], 'build', d['build']['ms'], 'probe', d['probe']['ms'])")" >> "$OUT/summary.txt"
  done
done
for g in 2 4; do
  timeout -k 10 300 python3 bench.py --gpus $g --rehearse --steps 20 --warmup 5 > "$OUT/gpus${g}_rehearsed.json" 2> "$OUT/gpus${g}_rehearsed.err" || exit 4
done
