#!/usr/bin/env bash
# Round-3 session N: kernel timelines (rocprofv3 --kernel-trace, per-launch
# start/end) of the strong-scaling shares issued by the native runner, to see
# where the N = 8 share (2 tables / 12.5 M lookups) loses time against linear:
# kernel durations vs gaps between kernels on each stream.
set -o pipefail
OUT=${1:-gpurun_out/r3n}
mkdir -p "$OUT"
export TMPDIR=/tmp
for share in "2 12500000 auto" "2 12500000 off" "16 100000000 auto"; do
  set -- $share
  tag=t$1_$3
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag" -o run -- \
    python3 bench.py --native --tables $1 --lookups $2 --overlap $3 --steps 30 --warmup 5 --no-cpu --no-e2e \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit 2
done
