# Version probe tiers with the sparse bound index (interleaved, one box):
# db_bench's version forced into each tier (DLSM_VERSION_LDS=1..5) with the
# current library, and the tree before the index ("pre", DLSM_VERSION_LDS=3
# / 4: the metadata-only and nothing-in-LDS tiers it replaces).
set -e
for r in 1 2; do
  for m in 1 2 3 4 5; do
    echo "== new DLSM_VERSION_LDS=$m round $r"
    DLSM_VERSION_LDS=$m timeout -k 10 200 python -u scripts/bench_version_probe.py --lookups 100000000 --check 0 --paths direct
  done
  for m in 3 4; do
    echo "== pre DLSM_VERSION_LDS=$m round $r"
    DLSM_LIB_VARIANT=pre DLSM_VERSION_LDS=$m timeout -k 10 200 python -u scripts/bench_version_probe.py --lookups 100000000 --check 0 --paths direct
  done
done
