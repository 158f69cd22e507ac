#!/usr/bin/env bash
# GPU parity tests, then bench A/B lines over scheduling knobs.
#   scripts/gpu_sweep.sh OUTDIR "label:bench args" ["label:bench args" ...]
# Each GPU step has its own time limit; the first failure ends the session.
set -o pipefail
OUT=${1:-gpurun_out/sweep}
shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || exit 1
for spec in "$@"; do
  label=${spec%%:*}
  args=${spec#*:}
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e $args \
    > "$OUT/bench_$label.json" 2> "$OUT/bench_$label.err" || exit 1
done
