#!/bin/bash
set -u
cd "$(dirname "$0")"
OUT=${GRAFT_REPO_ROOT:-../../..}/gpurun_out
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS}; do
    timeout -k 10 120 ./dec_ab_$v 262144 ${REPS:-3} >> "$OUT/dec_ab.log" 2>&1 || exit 1
  done
done
