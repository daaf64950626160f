#!/bin/bash
# encoder occupancy sweep on 1M chunks
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for w in ${WAVES:-16 24 32}; do
  NX_ENC_WAVES=$w timeout -k 10 240 python scripts/prof_encode.py 1048576 2 >> gpurun_out/enc_sweep.log 2>&1 || exit 1
done
