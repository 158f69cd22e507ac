# Version probe A/B (interleaved, one box): the current library ("new")
# against variants built with `make variant` (dlsm_amd/lib/variants/), direct
# path, 100 M Gets, no oracle check (tests/test_version_probe.py checks parity).
#   bash scripts/ab/version_variants_ab.sh ROUNDS VARIANT...
set -e
rounds=$1
shift
for r in $(seq 1 "$rounds"); do
  for v in new "$@"; do
    if [ "$v" = new ]; then unset DLSM_LIB_VARIANT; else export DLSM_LIB_VARIANT=$v; fi
    echo "== $v round $r"
    timeout -k 10 200 python -u scripts/bench_version_probe.py --lookups 100000000 --check 0 --paths direct
  done
done
