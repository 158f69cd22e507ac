# PMC passes over the version probe (scripts/bench_version_probe.py, direct,
# 100 M Gets), one counter group per rocprofv3 run, for the current library
# and an optional variant (DLSM_LIB_VARIANT); summaries only.
#   bash scripts/diag_version_pmc.sh OUTDIR [VARIANT]
set -e
OUT=$1
V=${2:-}
mkdir -p "$OUT"
i=0
# $VPMC_GROUPS: counter groups separated by ';' (default: fabric bytes and L2 hits)
IFS=';' read -r -a CGRPS <<< "${VPMC_GROUPS:-FETCH_SIZE;TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum}"
for grp in "${CGRPS[@]}"; do
  for lib in new $V; do
    i=$((i + 1))
    if [ "$lib" = new ]; then unset DLSM_LIB_VARIANT; else export DLSM_LIB_VARIANT=$lib; fi
    timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc$i/p1" -o run -- \
      python3 scripts/bench_version_probe.py --lookups 100000000 --check 0 --paths direct $VPMC_ARGS > "$OUT/p${i}_$lib.json" 2> "$OUT/p${i}_$lib.err"
    python3 scripts/pmc_summary.py "$OUT/pmc$i" 2>/dev/null | grep -A9 version_lds > "$OUT/p${i}_${lib}_summary.txt" || true
    rm -rf "$OUT/pmc$i"
  done
done
