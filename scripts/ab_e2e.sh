#!/bin/bash
# Alternate library builds on the end-to-end tool: VARIANTS="a b" FLUSHES="256 512" ROUNDS=2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS}; do
    for f in ${FLUSHES:-256 512}; do
      cp "netty_amd/build_variants/libnetty_amd_$v.so" netty_amd/libnetty_amd.so || exit 1
      echo -n "$v $f " >> gpurun_out/ab_e2e.log
      timeout -k 10 200 netty_amd/e2e_capi 256 256 65535 3 0 $f >> gpurun_out/ab_e2e.log 2>&1 || exit 1
    done
  done
done
