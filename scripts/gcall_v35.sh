# v35: round record (final tree of the session): full GPU suite, smoke, default bench (CPU baseline, e2e), 153,846-key SSTables,
# kernel traces, PMC FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
O=gpurun_out/v35
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --keys-per-table 153846 --no-e2e > $O/n153846.json 2> $O/n153846.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e > $O/bench_prof.json 2> $O/bench_prof.err &&
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" bash scripts/gpu_pmc.sh $O/pmc
