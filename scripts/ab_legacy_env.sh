#!/usr/bin/env bash
# Interleaved A/B of legacy-build env settings on scripts/bench_legacy.py,
# 3 rounds: each argument is one setting, "NAME=V[,NAME2=V2]" or "base".
#   bash scripts/ab_legacy_env.sh base DLSM_LEGACY_NC=0 ...
set -o pipefail
for r in 1 2 3; do
  for v in "$@"; do
    envs=""
    [ "$v" = base ] || envs=${v//,/ }
    env $envs timeout -k 10 120 python scripts/bench_legacy.py || exit 3
  done
done
