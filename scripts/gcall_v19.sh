# v19: parity + bench (default and 153,846-key SSTables) + kernel traces
set -o pipefail
O=gpurun_out/v19c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py --no-e2e > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --keys-per-table 153846 --no-e2e --steps 50 --warmup 10 > $O/n153846.json 2> $O/n153846.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $O/bench_prof.json 2> $O/bench_prof.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof153 -o run -- \
  python3 bench.py --keys-per-table 153846 --steps 10 --warmup 2 --no-cpu --no-e2e > $O/bench_prof153.json 2> $O/bench_prof153.err
