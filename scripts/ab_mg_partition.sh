# A/B of the one-pass probe's kernels: rocprofv3 kernel stats per library
# variant (DLSM_LIB_VARIANT tags, `make variant`) over the dedup-shifted and
# mixed filter sets at 100 M lookups.  bash scripts/ab_mg_partition.sh OUT TAG...
set -o pipefail
export TMPDIR=/tmp
O=${1:?out}
shift
mkdir -p $O
for v in "$@"; do
  if [ $v = base ]; then unset DLSM_LIB_VARIANT; else export DLSM_LIB_VARIANT=$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- python3 scripts/bench_probe_shapes.py --shapes dedup_shifted_8,mixed_8 --lookups 100000000 --reps 5 --check 0 --paths auto > $O/$v.log 2>&1 || exit 1
done
