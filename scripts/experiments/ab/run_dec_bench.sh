#!/bin/bash
# Alternating runs of Snappy decode builds (dec_bench_<v>), 262 144 frames, best of 3 per process.
set -u
cd "$(dirname "$0")"
OUT=${GRAFT_REPO_ROOT:-../../..}/gpurun_out
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS}; do
    echo -n "$v " >> "$OUT/dec_bench.log"
    timeout -k 10 120 ./dec_bench_$v 262144 3 1 >> "$OUT/dec_bench.log" 2>&1 || exit 1
  done
done
