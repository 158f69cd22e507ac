#!/usr/bin/env bash
# Round-3 session Y: 3-byte probe entries (sub-slice-ordered buckets, 12-byte
# units; DLSM_OPT_PROBE_ENTRY_BYTES default 3) -- the whole GPU suite first
# (every probe parity test runs the new default), then E3 vs 4-byte entries
# (DLSM_PROBE_ENTRY_BYTES=4) at the whole job and the N = 8 share, native
# runner, 100 steps, 3 interleaved rounds, and a kernel-trace of each.
set -o pipefail
OUT=${1:-gpurun_out/r3y}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || exit 2
for r in 1 2 3; do
  for share in "16 100000000" "2 12500000"; do
    set -- $share
    for eb in 3 4; do
      DLSM_PROBE_ENTRY_BYTES=$eb timeout -k 10 200 python3 bench.py --native --tables $1 --lookups $2 --steps 100 \
        --warmup 10 --no-cpu --no-e2e > "$OUT/t$1_e${eb}_$r.json" 2> "$OUT/t$1_e${eb}_$r.err" || exit 3
      echo "t$1 e$eb r$r $(python3 -c "import json; d=json.loads(open('$OUT/t$1_e${eb}_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'build', d['build']['ms'], 'probe', d['probe']['ms'])")" >> "$OUT/summary.txt"
    done
  done
done
for eb in 3 4; do
  DLSM_PROBE_ENTRY_BYTES=$eb timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_e$eb" -o run -- \
    python3 bench.py --native --overlap off --steps 40 --warmup 5 --no-cpu --no-e2e > "$OUT/prof_e$eb.json" 2> "$OUT/prof_e$eb.err" || exit 4
done
