#!/bin/bash
# Round 5 session 7: the segmented long-stream walk reworked (16-byte header loads, 4-wave guess with the
# whole first-hop rule in LDS, parallel straight-prefix stitch): frame-scan tests, timing against the
# lane walk on one ~1 GiB cumulation, kernel trace; then the whole -m gpu suite (NX_HIP_DEBUG=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s7
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_frame_scan.py \
    > $O/pytest_scan.log 2>&1; rc=$?; echo "pytest_scan $rc" >> $O/steps.log; fatal $rc pytest_scan; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/long_scan_prof.py 35840 5 > $O/long_scan.log 2>&1; rc=$?; echo "long_scan $rc" >> $O/steps.log; fatal $rc long_scan
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof_scan" -o run -- \
    python3 "$ROOT/scripts/long_scan_prof.py" 35840 5 > "$ROOT/$O/long_scan_prof.log" 2>&1); rc=$?; echo "prof_scan $rc" >> $O/steps.log; fatal $rc prof_scan
NX_HIP_DEBUG=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest_gpu $rc" >> $O/steps.log; fatal $rc pytest_gpu
exit 0
