# v27: 16,384-key probe chunks bucketed as two 8,192-key units (longer slice runs): parity, A/B vs 8,192
set -o pipefail
O=gpurun_out/v27
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_internal_keys.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
ROUNDS=3 bash scripts/gpu_ab.sh $O/ab "c13:DLSM_X=0|" "c14u:DLSM_X=0|--probe-chunk-lg 14" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof14 -o run -- \
  python3 bench.py --probe-chunk-lg 14 --steps 10 --warmup 2 --no-cpu --no-e2e > $O/bench_prof14.json 2> $O/bench_prof14.err
