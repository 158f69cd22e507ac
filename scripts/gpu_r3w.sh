#!/usr/bin/env bash
# Round-3 session W: scheduling of the overlapped step.  new = the probe slice
# pass's image in dynamic LDS sized to the slice (245 lines: 26 KiB of the CU
# free, room for a build partition workgroup beside it); old = the static
# 256-line array (variant); bap = the build issued behind the probe's
# partition pass (DLSM_STEP_BUILD_AFTER_PARTITION, dlsm_ctx_set_partition_event);
# prio = the probe stream at the higher priority.  Parity tests first; native
# runner, 100 steps, 3 interleaved rounds; timelines of new and bap.
set -o pipefail
OUT=${1:-gpurun_out/r3w}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_walk_edges.py tests/test_gpu_packed_groups.py tests/test_gpu_fullsize.py > "$OUT/pytest.log" 2>&1 || exit 2
for r in 1 2 3; do
  for share in "16 100000000" "2 12500000"; do
    set -- $share
    for spec in "old:DLSM_LIB_VARIANT=old" "new:X=0" "bap:DLSM_STEP_BUILD_AFTER_PARTITION=1" \
                "bapold:DLSM_LIB_VARIANT=old DLSM_STEP_BUILD_AFTER_PARTITION=1" "prio:DLSM_BENCH_PROBE_PRIORITY=-1"; do
      label=${spec%%:*}; envs=${spec#*:}
      env $envs timeout -k 10 200 python3 bench.py --native --tables $1 --lookups $2 --steps 100 --warmup 10 \
        --no-cpu --no-e2e > "$OUT/t$1_${label}_$r.json" 2> "$OUT/t$1_${label}_$r.err" || exit 3
      echo "t$1 $label r$r $(python3 -c "import json; d=json.loads(open('$OUT/t$1_${label}_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'build', d['build']['ms'], 'probe', d['probe']['ms'])")" >> "$OUT/summary.txt"
    done
  done
done
for spec in "new:X=0" "bap:DLSM_STEP_BUILD_AFTER_PARTITION=1"; do
  label=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl_$label" -o run -- \
    python3 bench.py --native --steps 40 --warmup 5 --no-cpu --no-e2e > "$OUT/tl_$label.json" 2> "$OUT/tl_$label.err" || exit 4
done
