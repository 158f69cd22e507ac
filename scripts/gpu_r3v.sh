#!/usr/bin/env bash
# Round-3 session V: build beside probe on two streams at every N (overlap
# auto = on), the sampled steps running their passes alone; GPU tests of the
# runner / bench paths, then default vs --overlap off at the whole job and
# the N = 8 share (native runner and Python loop), 3 interleaved rounds.
set -o pipefail
OUT=${1:-gpurun_out/r3v}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_multigpu_threads.py \
  tests/test_multirank.py tests/test_bench_contract.py > "$OUT/pytest.log" 2>&1 || exit 2
for r in 1 2 3; do
  for spec in "t16:--tables 16 --lookups 100000000" "t2:--tables 2 --lookups 12500000 --native" "py16:--python-loop"; do
    label=${spec%%:*}; a=${spec#*:}
    for ov in auto off; do
      timeout -k 10 200 python3 bench.py $a --overlap $ov --steps 100 --warmup 10 --no-cpu --no-e2e \
        > "$OUT/${label}_${ov}_$r.json" 2> "$OUT/${label}_${ov}_$r.err" || exit 3
      echo "$label $ov r$r $(python3 -c "import json; d=json.loads(open('$OUT/${label}_${ov}_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'build', d['build']['ms'], 'probe', d['probe']['ms'], 'frac', d['roofline']['frac'], 'step_frac', d['roofline']['step_frac'])")" >> "$OUT/summary.txt"
    done
  done
done
timeout -k 10 400 python3 bench.py > "$OUT/bench_full.json" 2> "$OUT/bench_full.err" || exit 4
