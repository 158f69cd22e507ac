#!/usr/bin/env bash
# Round-3 session X: the launcher path (torch.distributed.run, one process per
# GPU) timed by the native runner: the runner / bench GPU tests, and a 2-rank
# gloo rehearsal of the driver's N = 2 command on the one GPU.
set -o pipefail
OUT=${1:-gpurun_out/r3x}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multigpu_threads.py \
  tests/test_multirank.py > "$OUT/pytest.log" 2>&1 || exit 2
DLSM_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
  > "$OUT/launcher_gpus2_rehearsed.json" 2> "$OUT/launcher_gpus2_rehearsed.err" || exit 3
