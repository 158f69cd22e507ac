#!/usr/bin/env bash
# Round-3 session P: pass events sampled on 4 of the timed steps (native
# runner and Python loops): GPU tests of the runner, timelines of the t2 share
# and the whole job without per-step events, bench lines.
set -o pipefail
OUT=${1:-gpurun_out/r3p}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_multigpu_threads.py \
  tests/test_multirank.py > "$OUT/pytest.log" 2>&1 || exit 2
for share in "2 12500000" "16 100000000"; do
  set -- $share
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl_t$1" -o run -- \
    python3 bench.py --native --tables $1 --lookups $2 --steps 40 --warmup 5 --no-cpu --no-e2e \
    > "$OUT/tl_t$1.json" 2> "$OUT/tl_t$1.err" || exit 3
done
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 100 --warmup 10 --no-cpu --no-e2e > "$OUT/bench_$r.json" 2> "$OUT/bench_$r.err" || exit 4
  timeout -k 10 200 python3 bench.py --native --tables 2 --lookups 12500000 --steps 100 --warmup 10 --no-cpu --no-e2e \
    > "$OUT/t2_$r.json" 2> "$OUT/t2_$r.err" || exit 5
  timeout -k 10 200 python3 bench.py --python-loop --steps 100 --warmup 10 --no-cpu --no-e2e > "$OUT/pyloop_$r.json" 2> "$OUT/pyloop_$r.err" || exit 6
done
