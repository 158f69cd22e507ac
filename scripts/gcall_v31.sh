# v31: 8,192-key probe chunks as two 4,096-key units in 512-thread workgroups (two resident per CU,
# partition phases interleave) vs the 16,384-key default
set -o pipefail
O=gpurun_out/v31
mkdir -p $O
export TMPDIR=/tmp
DLSM_LIB_VARIANT=p13 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k probe --timeout 120 --timeout-method thread > $O/pytest_p13.log 2>&1 &&
ROUNDS=3 bash scripts/gpu_ab.sh $O/ab "c14:DLSM_X=0|" "p13:DLSM_LIB_VARIANT=p13|--probe-chunk-lg 13" "c13:DLSM_X=0|--probe-chunk-lg 13" &&
DLSM_LIB_VARIANT=p13 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_p13 -o run -- \
  python3 bench.py --probe-chunk-lg 13 --steps 10 --warmup 2 --no-cpu --no-e2e > $O/bench_prof.json 2> $O/bench_prof.err
