#!/bin/bash
# Round 5 session 20: kernel trace of the alt-codec leg (FastLZ L1/L2, LZF, LZ4; 262 144 mixed blocks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s20
mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof" -o run -- \
    python3 "$ROOT/scripts/alt_traffic_run.py" 262144 > "$ROOT/$O/prof.log" 2>&1); rc=$?; echo "prof $rc" >> $O/steps.log
exit 0
