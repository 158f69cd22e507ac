# v20: re-verify the rebuilt tree: parity, smoke, bench, kernel traces
set -o pipefail
O=gpurun_out/v20
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $O/bench_prof.json 2> $O/bench_prof.err
