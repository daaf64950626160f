#!/bin/bash
# Alternate library builds (netty_amd/build_variants/libnetty_amd_<v>.so) on the Snappy decode timing
# of scripts/dec_time.py (262144 text frames, parse + expand + CRC verify).  VARIANTS="a b" ROUNDS=3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS}; do
    cp "netty_amd/build_variants/libnetty_amd_$v.so" netty_amd/libnetty_amd.so || exit 1
    echo -n "$v " >> gpurun_out/ab_dec.log
    timeout -k 10 200 python scripts/dec_time.py ${N:-262144} ${REPS:-5} >> gpurun_out/ab_dec.log 2>&1 || exit 1
  done
done
