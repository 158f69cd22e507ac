#!/usr/bin/env bash
# Interleaved A/B of how host-API calls wait for the GPU (DLSM_HOST_SYNC:
# 0 hipStreamSynchronize, 1 event poll + sched_yield, 2 blocking-sync event)
# on tests/cpp/concurrent_builders: ROUNDS rounds x modes x thread counts.
#   bash scripts/ab_builders_sync.sh OUT.jsonl CB_BINARY [ROUNDS] [THREADS] [MODES] [SYNCS]
set -o pipefail
out=${1:?out}; cb=${2:?cb}; rounds=${3:-3}; threads=${4:-16,28}; modes=${5:-ref,hash}; syncs=${6:-0,1,2}
for r in $(seq 1 "$rounds"); do
  for sy in ${syncs//,/ }; do
    for mode in ${modes//,/ }; do
      for t in ${threads//,/ }; do
        DLSM_HOST_SYNC=$sy timeout -k 10 180 "$cb" "$t" 8 153846 "$mode" >> "$out" || exit 3
      done
    done
  done
done
