# v29: unit loop not unrolled (14 vs 21 VGPR spills) vs unrolled ("unr" = HEAD)
set -o pipefail
O=gpurun_out/v29
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k probe --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
ROUNDS=4 bash scripts/gpu_ab.sh $O/ab "unr:DLSM_LIB_VARIANT=unr|" "nounroll:DLSM_X=0|"
