#!/bin/bash
# End-to-end tool at several event-loop thread counts (one batcher per thread): THREADS="1 2 4"
# FLUSH=256 ROUNDS=2.  Output: gpurun_out/e2e_threads.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for t in ${THREADS:-1 2 4}; do
    for f in ${FLUSH:-256}; do
      echo -n "T$t F$f " >> gpurun_out/e2e_threads.log
      timeout -k 10 240 netty_amd/e2e_capi 256 256 65535 3 0 $f $t >> gpurun_out/e2e_threads.log 2>&1 || exit 1
    done
  done
done
