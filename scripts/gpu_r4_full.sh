#!/bin/bash
# Round-4 evidence session: smoke, the driver's default bench line, a rocprofv3 kernel trace of
# the bench workload at 262 144 chunks per dispatch, and the FETCH/WRITE traffic passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
CHUNKS=262144 STAGE=smoke bash scripts/gpu_round.sh || exit 1
CHUNKS=262144 STAGE=full bash scripts/gpu_round.sh || exit 1
CHUNKS=262144 STAGE=prof bash scripts/gpu_round.sh || exit 1
CHUNKS=262144 STAGE=pmc bash scripts/gpu_round.sh || exit 1
