#!/usr/bin/env bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only; no
# sys/runtime traces beside --pmc).  FETCH_SIZE and WRITE_SIZE in separate
# passes (TCC slot limits, MI355X_MICROARCH.md §rocprofv3 PMC slots).
#   BENCH_ARGS="..." scripts/gpu_pmc.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-e2e ${BENCH_ARGS:-}"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
# PMC_GROUPS: ';'-separated counter groups replacing the default ones
IFS=';' read -r -a PMC_GRPS <<< "${PMC_GROUPS:-FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS;SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum}"
for grp in "${PMC_GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
    $BENCH > "$OUT/p$i.json" 2> "$OUT/p$i.err" || exit 1
done
