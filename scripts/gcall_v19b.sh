set -o pipefail
O=gpurun_out/v19b
mkdir -p $O
ROUNDS=3 timeout -k 10 900 bash scripts/gpu_ab.sh $O/ab "gs:X=1|" "gs64:DLSM_LIB_VARIANT=gs64|"
