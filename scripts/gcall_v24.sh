# v24: build partition with all key tiles of a chunk in flight at once (DLSM_TILE_ALL) vs one tile
# ahead ("base"), and 2,048-key build chunks ("c2k"); bench and 153,846-key SSTables, interleaved
set -o pipefail
O=gpurun_out/v24
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_internal_keys.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
DLSM_LIB_VARIANT=c2k timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_c2k.log 2>&1 &&
ROUNDS=3 bash scripts/gpu_ab.sh $O/ab "base:DLSM_LIB_VARIANT=base|" "all:DLSM_X=0|" "c2k:DLSM_LIB_VARIANT=c2k|" \
  "base153:DLSM_LIB_VARIANT=base|--keys-per-table 153846" "all153:DLSM_X=0|--keys-per-table 153846" "c2k153:DLSM_LIB_VARIANT=c2k|--keys-per-table 153846"
