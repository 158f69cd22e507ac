#!/usr/bin/env bash
# rocprofv3 kernel-trace summaries of short bench runs, one per labelled
# spec "label:ENV=.. ENV2=..|bench args" (no PMC): per-kernel average
# durations for A/B work.
#   scripts/gpu_kprof.sh OUTDIR spec ...
set -o pipefail
OUT=${1:-gpurun_out/kprof}
shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  label=${spec%%:*}
  rest=${spec#*:}
  envs=${rest%%|*}
  args=${rest#*|}
  mkdir -p "$OUT/$label"
  for e in $envs; do export "$e"; done
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$label" -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e $args \
    > "$OUT/$label/bench.json" 2> "$OUT/$label.err" || exit 1
  for e in $envs; do unset "${e%%=*}"; done
done
