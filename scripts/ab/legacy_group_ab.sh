set -e
for r in 1 2; do
  for g in 160 0; do
    echo "== DLSM_LEGACY_GROUP_MB=$g round $r"
    DLSM_LEGACY_GROUP_MB=$g timeout -k 10 200 python -u bench.py --no-cpu --no-e2e --no-version --no-mixed --steps 20
  done
done
