# v25: build partition issues the dedup-neighbour hash before the tile loads; A/B vs HEAD ("base")
set -o pipefail
O=gpurun_out/v25
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_internal_keys.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
ROUNDS=4 bash scripts/gpu_ab.sh $O/ab "base:DLSM_LIB_VARIANT=base|" "prev:DLSM_X=0|" \
  "base153:DLSM_LIB_VARIANT=base|--keys-per-table 153846" "prev153:DLSM_X=0|--keys-per-table 153846" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof153 -o run -- \
  python3 bench.py --keys-per-table 153846 --steps 10 --warmup 2 --no-cpu --no-e2e > $O/bench_prof153.json 2> $O/bench_prof153.err
