# Version probe tiers whose file metadata is read from global memory
# (DLSM_VERSION_LDS=4: sparse bound index only; =5: nothing in LDS), current
# library vs "pre" (the tree before), interleaved on one box.
set -e
for r in 1 2 3; do
  for v in new pre; do
    for m in 4 5; do
      echo "== $v DLSM_VERSION_LDS=$m round $r"
      if [ "$v" = new ]; then unset DLSM_LIB_VARIANT; else export DLSM_LIB_VARIANT=$v; fi
      DLSM_VERSION_LDS=$m timeout -k 10 200 python -u scripts/bench_version_probe.py --lookups 100000000 --check 0 --paths direct
    done
  done
done
