#!/usr/bin/env bash
# Interleaved A/B bench lines on one box: each "label:ENV=.. ENV2=..|bench args"
# spec runs ROUNDS times, alternating, so box-to-box variance cancels.
#   ROUNDS=3 scripts/gpu_ab.sh OUTDIR spec...
set -o pipefail
OUT=${1:-gpurun_out/ab}
shift || true
mkdir -p "$OUT"
for r in $(seq 1 "${ROUNDS:-3}"); do
  for spec in "$@"; do
    label=${spec%%:*}
    rest=${spec#*:}
    envs=${rest%%|*}
    args=${rest#*|}
    env $envs timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --no-legacy $args \
      > "$OUT/${label}_$r.json" 2> "$OUT/${label}_$r.err" || exit 1
  done
done
