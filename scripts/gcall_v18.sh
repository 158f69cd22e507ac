set -o pipefail
O=gpurun_out/v18
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err &&
ROUNDS=2 timeout -k 10 600 bash scripts/gpu_ab.sh $O/ab "c13:X=1|--probe-chunk-lg 13" "c14:X=1|--probe-chunk-lg 14"
