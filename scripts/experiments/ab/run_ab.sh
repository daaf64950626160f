#!/bin/bash
# Same-box A/B of encoder builds (enc_ab_<v> for v in $VARIANTS), alternating, 262 144 chunks.
set -u
cd "$(dirname "$0")"
OUT=${GRAFT_REPO_ROOT:-../../..}/gpurun_out
mkdir -p "$OUT"
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-a b}; do
    timeout -k 10 120 ./enc_ab_$v 262144 ${REPS:-3} >> "$OUT/ab.log" 2>&1 || exit 1
  done
done
