#!/usr/bin/env bash
# Round-3 session A: GPU parity tests, the default bench line, and the
# one-process multi-GPU bench rehearsed on the box's one GPU (2 and 4 logical
# devices).  Each GPU step has its own limit.  Test failures (pytest rc 1)
# still let the benches run; anything else (a crash, a time limit) ends it.
set -o pipefail
OUT=${1:-gpurun_out/r3a}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 python bench.py --gpus 2 --rehearse --steps 20 --warmup 5 > "$OUT/bench_g2r.json" 2> "$OUT/bench_g2r.err" &&
timeout -k 10 300 python bench.py --gpus 4 --rehearse --steps 20 --warmup 5 > "$OUT/bench_g4r.json" 2> "$OUT/bench_g4r.err" &&
timeout -k 10 300 python tests/diag/run_scatter_mask.py > "$OUT/scatter_mask.json" 2> "$OUT/scatter_mask.err" &&
exit $rc
