#!/usr/bin/env bash
# One GPU session: parity tests, a profiled bench, and probe-round A/B.
# Every GPU step has its own time limit and the steps are chained with &&.
set -o pipefail
OUT=${1:-gpurun_out/run}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" &&
for r in ${ROUNDS:-}; do
  DLSM_PROBE_ROUND_KEYS=$r timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-e2e \
    > "$OUT/bench_round_$r.json" 2> "$OUT/bench_round_$r.err" || exit 1
done
