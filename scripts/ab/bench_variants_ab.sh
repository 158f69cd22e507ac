# bench.py A/B over library variants (interleaved, one box): the current
# library ("new") against variants built with `make variant`.
#   bash scripts/ab/bench_variants_ab.sh ROUNDS "BENCH ARGS" VARIANT...
set -e
rounds=$1
bargs=$2
shift 2
for r in $(seq 1 "$rounds"); do
  for v in new "$@"; do
    if [ "$v" = new ]; then unset DLSM_LIB_VARIANT; else export DLSM_LIB_VARIANT=$v; fi
    echo "== $v round $r"
    timeout -k 10 300 python -u bench.py $bargs
  done
done
