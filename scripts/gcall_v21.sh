# v21: slice-byte (DLSM_PROBE_SB) variant: parity of the probe tests, then interleaved A/B
set -o pipefail
O=gpurun_out/v21
mkdir -p $O
export TMPDIR=/tmp
DLSM_LIB_VARIANT=sb timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_sb.log 2>&1 &&
ROUNDS=4 bash scripts/gpu_ab.sh $O/ab "base:DLSM_X=0|" "sb:DLSM_LIB_VARIANT=sb|" &&
DLSM_LIB_VARIANT=sb timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sb -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $O/bench_prof_sb.json 2> $O/bench_prof_sb.err
