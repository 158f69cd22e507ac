# v22: build slice with straight-line k = 6 bit-sets: parity, interleaved A/B vs the v20 code (variant "base")
set -o pipefail
O=gpurun_out/v22
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
ROUNDS=4 bash scripts/gpu_ab.sh $O/ab "base:DLSM_LIB_VARIANT=base|" "k6:DLSM_X=0|" "base153:DLSM_LIB_VARIANT=base|--keys-per-table 153846" "k6153:DLSM_X=0|--keys-per-table 153846" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $O/bench_prof.json 2> $O/bench_prof.err
