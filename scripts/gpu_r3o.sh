#!/usr/bin/env bash
# Round-3 session O: do the per-pass HIP events inside the timed loop cost
# step time?  Native runner, events on (default) vs off (DLSM_NO_PASS_EVENTS=1),
# whole job (t16) and the N = 8 share (t2), 3 interleaved rounds, 100 steps.
set -o pipefail
OUT=${1:-gpurun_out/r3o}
mkdir -p "$OUT"
for r in 1 2 3; do
  for share in "16 100000000" "2 12500000" "4 25000000"; do
    set -- $share
    for ev in 0 1; do
      DLSM_NO_PASS_EVENTS=$ev timeout -k 10 200 python3 bench.py --native --tables $1 --lookups $2 --steps 100 --warmup 10 \
        --no-cpu --no-e2e > "$OUT/t$1_ev${ev}_$r.json" 2> "$OUT/t$1_ev${ev}_$r.err" || exit 2
      echo "t$1 noev=$ev round $r $(python3 -c "import json,sys; d=json.loads(open('$OUT/t$1_ev${ev}_$r.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])")" >> "$OUT/summary.txt"
    done
  done
done
