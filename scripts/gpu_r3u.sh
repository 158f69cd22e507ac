#!/usr/bin/env bash
# Round-3 session U: build beside probe on two streams (--overlap on) vs one
# stream (off) at the whole job, now that the timed steps carry no per-step
# events; N = 2 share for reference.  Native runner, 100 steps, 4 interleaved
# rounds.
set -o pipefail
OUT=${1:-gpurun_out/r3u}
mkdir -p "$OUT"
for r in 1 2 3 4; do
  for share in "16 100000000" "8 50000000"; do
    set -- $share
    for ov in off on; do
      timeout -k 10 200 python3 bench.py --native --tables $1 --lookups $2 --overlap $ov --steps 100 --warmup 10 \
        --no-cpu --no-e2e > "$OUT/t$1_${ov}_$r.json" 2> "$OUT/t$1_${ov}_$r.err" || exit 2
      echo "t$1 $ov r$r $(python3 -c "import json; d=json.loads(open('$OUT/t$1_${ov}_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'build', d['build']['ms'], 'probe', d['probe']['ms'])")" >> "$OUT/summary.txt"
    done
  done
done
