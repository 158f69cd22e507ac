#!/usr/bin/env bash
# Round-3 session AD: the persistent, tile-pipelined build partition
# (full_partition_pipe_kernel, DLSM_BUILD_PIPE=1) vs one workgroup per chunk.
# Build parity tests with the pipe kernel first; native runner, 100 steps, 3
# interleaved rounds at the whole job and the N = 2 / 4 / 8 shares; kernel
# stats of the N = 8 share with overlap off.
set -o pipefail
OUT=${1:-gpurun_out/r3ad}
mkdir -p "$OUT"
export TMPDIR=/tmp
DLSM_BUILD_PIPE=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_workspace.py tests/test_gpu_hashed_build.py \
  tests/test_internal_keys.py tests/test_gpu_adapter.py tests/test_multigpu_threads.py > "$OUT/pytest.log" 2>&1 || exit 2
for r in 1 2 3; do
  for share in "16 100000000" "4 25000000" "2 12500000"; do
    set -- $share
    for p in 0 1; do
      DLSM_BUILD_PIPE=$p timeout -k 10 200 python3 bench.py --native --tables $1 --lookups $2 --steps 100 --warmup 10 \
        --no-cpu --no-e2e > "$OUT/t$1_p${p}_$r.json" 2> "$OUT/t$1_p${p}_$r.err" || exit 3
      echo "t$1 pipe$p r$r $(python3 -c "import json; d=json.loads(open('$OUT/t$1_p${p}_$r.json').read().strip().splitlines()[-1]); print('ms_per_step', d['ms_per_step'], 'build', d['build']['ms'], 'probe', d['probe']['ms'])")" >> "$OUT/summary.txt"
    done
  done
done
for p in 0 1; do
  DLSM_BUILD_PIPE=$p timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_t2_p$p" -o run -- \
    python3 bench.py --native --tables 2 --lookups 12500000 --overlap off --steps 40 --warmup 5 --no-cpu --no-e2e \
    > "$OUT/prof_t2_p$p.json" 2> "$OUT/prof_t2_p$p.err" || exit 4
  DLSM_BUILD_PIPE=$p timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_t16_p$p" -o run -- \
    python3 bench.py --native --overlap off --steps 20 --warmup 5 --no-cpu --no-e2e \
    > "$OUT/prof_t16_p$p.json" 2> "$OUT/prof_t16_p$p.err" || exit 4
done
