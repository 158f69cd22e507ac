#!/usr/bin/env bash
# Final confirmation on the round's last tree: the whole GPU suite, smoke, the
# default bench line (what the driver runs at round end).
set -o pipefail
OUT=${1:-gpurun_out/final}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
