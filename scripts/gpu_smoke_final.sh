#!/usr/bin/env bash
# Last check of the in-tree binaries: smoke + the runner/bench GPU tests + a short default bench.
set -o pipefail
OUT=${1:-gpurun_out/smoke_final}
mkdir -p "$OUT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_multigpu_threads.py \
  tests/test_gpu_fullsize.py > "$OUT/pytest.log" 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e > "$OUT/bench.json" 2> "$OUT/bench.err"
