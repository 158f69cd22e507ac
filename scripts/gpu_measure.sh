#!/usr/bin/env bash
# One measuring GPU session: parity tests, rocprofv3 PMC passes (one counter
# group per run, --kernel-trace only) -> per-launch traffic summary, the full
# bench line (cpu_baseline + e2e + traffic), and a rocprofv3 kernel-trace
# --stats summary of the same bench command, with the kernels of the steps
# whose passes the bench times (scripts/sampled_kernel_stats.py).  Each GPU step has its own time
# limit; the steps are chained with && so the first failure ends the session.
#   scripts/gpu_measure.sh OUTDIR [extra bench args...]
set -o pipefail
OUT=${1:-gpurun_out/measure}
shift || true
mkdir -p "$OUT"
export TMPDIR=/tmp
BARGS="$*"
# SKIP_TESTS=1: the parity suite ran in an earlier call on the same tree
{ [ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; } &&
timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
i=0 &&
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  mkdir -p "$OUT/pmc" &&
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc/p$i" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --no-version --no-mixed --no-block $BARGS \
    > "$OUT/pmc/p$i.json" 2> "$OUT/pmc/p$i.err" || exit 1
done &&
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  mkdir -p "$OUT/pmcv" &&
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmcv/p$i" -o run -- \
    python3 scripts/bench_version_probe.py --lookups 100000000 --check 0 --paths direct \
    > "$OUT/pmcv/p$i.json" 2> "$OUT/pmcv/p$i.err" || exit 1
done &&
for shape in mixed_set dedup_shifted; do
  for grp in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    mkdir -p "$OUT/pmc_$shape" &&
    timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc_$shape/p$i" -o run -- \
      python3 scripts/bench_probe_shapes.py --shapes $shape --lookups 100000000 --reps 3 --check 0 --paths auto \
      > "$OUT/pmc_$shape/p$i.json" 2> "$OUT/pmc_$shape/p$i.err" || exit 1
  done
done &&
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  mkdir -p "$OUT/pmc_block" &&
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc_block/p$i" -o run -- \
    python3 scripts/bench_block.py --only-block --reps 3 \
    > "$OUT/pmc_block/p$i.json" 2> "$OUT/pmc_block/p$i.err" || exit 1
done &&
python3 scripts/pmc_traffic.py "$OUT/pmc" "$OUT/pmc/p1.json" "$OUT/traffic.json" "$OUT/pmcv" \
  mixed_set="$OUT/pmc_mixed_set" dedup_shifted="$OUT/pmc_dedup_shifted" block="$OUT/pmc_block" > /dev/null &&
timeout -k 10 400 python bench.py --traffic "$OUT/traffic.json" $BARGS > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-legacy --no-version --no-mixed --no-block \
  --traffic "$OUT/traffic.json" $BARGS > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" &&
python3 scripts/sampled_kernel_stats.py "$OUT/prof" 10 > "$OUT/sampled_kernel_stats.txt" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/vprof" -o run -- \
  python3 scripts/bench_version_probe.py --lookups 100000000 --check 0 --paths direct \
  > "$OUT/vprof.json" 2> "$OUT/vprof.err" &&
python3 scripts/kstats.py "$OUT/vprof" > "$OUT/version_kernel_stats.txt" 2>&1 &&
python3 scripts/shrink_outputs.py "$OUT"
