# Probe slice shape at the N = 8 and N = 4 shares (interleaved, one box):
# 128 KiB slices (default) vs 64 KiB slices, each with the automatic part
# count and with one part per slice.  Prints each run's bench line.
#   bash scripts/ab/share_slice_shape_ab.sh ROUNDS
set -e
rounds=$1
common="--steps 200 --warmup 20 --no-cpu --no-e2e --no-legacy --no-version --no-mixed --native"
for r in $(seq 1 "$rounds"); do
  for share in "2 12500000" "4 25000000"; do
    set -- $share
    for shape in "8 0" "7 0" "8 1" "7 1"; do
      set -- $share $shape
      echo "== tables $1 lookups $2 slice_lg $3 parts $4 round $r"
      if [ "$4" = 0 ]; then unset DLSM_SLICE_PARTS; else export DLSM_SLICE_PARTS=$4; fi
      timeout -k 10 200 python -u bench.py --tables $1 --lookups $2 --probe-slice-lg $3 $common
    done
  done
done
