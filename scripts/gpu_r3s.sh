#!/usr/bin/env bash
# Round-3 session S: issue order of a step's two calls on their two streams at
# the shares (DLSM_STEP_PROBE_FIRST=1: probe then build; default: build then
# probe), native runner, 100 steps, 3 interleaved rounds; plus a kernel
# timeline of the N = 8 share in each order.
set -o pipefail
OUT=${1:-gpurun_out/r3s}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2 3; do
  for share in "2 12500000" "4 25000000" "16 100000000"; do
    set -- $share
    for pf in 0 1; do
      DLSM_STEP_PROBE_FIRST=$pf timeout -k 10 200 python3 bench.py --native --tables $1 --lookups $2 --steps 100 --warmup 10 \
        --no-cpu --no-e2e > "$OUT/t$1_pf${pf}_$r.json" 2> "$OUT/t$1_pf${pf}_$r.err" || exit 2
      echo "t$1 pf$pf r$r $(python3 -c "import json; d=json.loads(open('$OUT/t$1_pf${pf}_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'build', d['build']['ms'], 'probe', d['probe']['ms'])")" >> "$OUT/summary.txt"
    done
  done
done
for pf in 0 1; do
  DLSM_STEP_PROBE_FIRST=$pf timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl_pf$pf" -o run -- \
    python3 bench.py --native --tables 2 --lookups 12500000 --steps 40 --warmup 5 --no-cpu --no-e2e \
    > "$OUT/tl_pf$pf.json" 2> "$OUT/tl_pf$pf.err" || exit 3
done
