#!/bin/bash
# Round 5 session 1: encoder insert-store A/B (placement-controlled) and decode latency by batch size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s1
mkdir -p $O
timeout -k 10 400 ./scripts/experiments/bin/enc_ab3_plain 262144 4 > $O/enc_ab_plain.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/dec_latency.py 3 > $O/dec_latency.log 2>&1 || exit 2
