# PMC passes (one counter group per run) over the one-pass multi-group probe:
# bench_probe_shapes.py on one shape, 100 M lookups, auto path only.
#   bash scripts/diag_mg_pmc.sh OUT SHAPE
set -o pipefail
export TMPDIR=/tmp
O=${1:?out}
SHAPE=${2:-dedup_shifted_8}
mkdir -p $O
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/p$i -o run -- \
    python3 scripts/bench_probe_shapes.py --shapes $SHAPE --lookups 100000000 --reps 2 --check 0 --paths auto \
    > $O/p$i.log 2>&1 || exit 1
done
