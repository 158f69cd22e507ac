# v34: build entries carry the line offset (no fastmod in the build slice pass) vs fastmod ("fm")
set -o pipefail
O=gpurun_out/v34
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
ROUNDS=4 bash scripts/gpu_ab.sh $O/ab "fm:DLSM_LIB_VARIANT=fm|" "line:DLSM_X=0|" "fm153:DLSM_LIB_VARIANT=fm|--keys-per-table 153846" "line153:DLSM_X=0|--keys-per-table 153846" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $O/bench_prof.json 2> $O/bench_prof.err
