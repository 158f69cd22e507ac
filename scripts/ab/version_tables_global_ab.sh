# Version probe (db_bench shape, direct, 100 M Gets) with its tables in LDS
# (DLSM_VERSION_LDS=1, the default for <= ~450 files), bound prefixes only in
# LDS (=2, the tier for <= ~1,800 files) and all tables in global memory (=3),
# interleaved on one box.
set -e
for r in 1 2; do
  for m in 1 2 3; do
    echo "== DLSM_VERSION_LDS=$m round $r"
    DLSM_VERSION_LDS=$m timeout -k 10 200 python -u scripts/bench_version_probe.py --lookups 100000000 --check 0 --paths direct
  done
done
