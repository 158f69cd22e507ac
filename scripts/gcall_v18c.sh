# v18c: kernel trace of the 153,846-key SSTable variant
set -o pipefail
O=gpurun_out/v18c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --keys-per-table 153846 --steps 10 --warmup 2 --no-cpu --no-e2e > $O/bench.json 2> $O/bench.err
