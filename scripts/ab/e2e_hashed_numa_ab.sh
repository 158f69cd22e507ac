# e2e_hashed with the host-hash pool NUMA-placed (default) vs left anywhere
# (DLSM_HASH_NUMA=0), interleaved on one box; prints the e2e_hashed record.
set -e
for r in 1 2; do
  for v in 1 0; do
    echo "== DLSM_HASH_NUMA=$v round $r"
    DLSM_HASH_NUMA=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --no-legacy --no-version --no-mixed \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps(d['e2e_hashed']))"
  done
done
