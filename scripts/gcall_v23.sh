# v23: K28 LDS-tiled loaders for 28-byte internal keys: full GPU suite, internal-key rates vs the
# generic loader (variant "base" = v22 code), default bench A/B (K20 path unchanged)
set -o pipefail
O=gpurun_out/v23
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python scripts/bench_internal_keys.py > $O/internal_k28.json 2> $O/internal_k28.err &&
DLSM_LIB_VARIANT=base timeout -k 10 300 python scripts/bench_internal_keys.py > $O/internal_base.json 2> $O/internal_base.err &&
ROUNDS=3 bash scripts/gpu_ab.sh $O/ab "base:DLSM_LIB_VARIANT=base|" "k28:DLSM_X=0|"
