# Version probe (db_bench shape, direct, 100 M Gets) by how much of its tables
# the LDS holds (DLSM_VERSION_LDS=1: all, the default up to ~440 files; =2:
# file metadata + bound prefixes, the tier up to ~770 files; =3: the
# metadata, up to ~1,500; =4: none), interleaved on one box.
set -e
for r in 1 2; do
  for m in 1 2 3 4; do
    echo "== DLSM_VERSION_LDS=$m round $r"
    DLSM_VERSION_LDS=$m timeout -k 10 200 python -u scripts/bench_version_probe.py --lookups 100000000 --check 0 --paths direct
  done
done
