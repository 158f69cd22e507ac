# v28: probe slice walk sweep (windows per wave U8, walk depth) at 16,384-key unit-split chunks
set -o pipefail
O=gpurun_out/v28
mkdir -p $O
export TMPDIR=/tmp
DLSM_LIB_VARIANT=d2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k probe --timeout 120 --timeout-method thread > $O/pytest_d2.log 2>&1 &&
ROUNDS=3 bash scripts/gpu_ab.sh $O/ab "c14u:DLSM_X=0|--probe-chunk-lg 14" "u4:DLSM_LIB_VARIANT=u4|--probe-chunk-lg 14" \
  "u3:DLSM_LIB_VARIANT=u3|--probe-chunk-lg 14" "d2:DLSM_LIB_VARIANT=d2|--probe-chunk-lg 14" "c13:DLSM_X=0|"
