#!/bin/bash
# Round 6 session 1: encoder time against chunks per launch, placement-
# controlled (A = product kernel: 32-dword stage, 4 blocks per CU; B = 16-dword stage, 5 blocks per
# CU), and Snappy decode + verify time against frames per call, with a kernel trace of the latter.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r6s1
mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
timeout -k 10 300 scripts/experiments/bin/enc_curve_s16lb5 2 32768 65536 131072 163840 196608 204800 229376 262144 273152 294912 327680 \
    > $O/enc_curve.log 2>&1; rc=$?; echo "enc_curve $rc" >> $O/steps.log; fatal $rc enc_curve
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof" -o run -- \
    python3 "$ROOT/scripts/dec_curve.py" 3 65536 131072 163840 204800 262144 327680 > "$ROOT/$O/dec_curve.log" 2>&1); rc=$?
echo "dec_curve $rc" >> $O/steps.log
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1); [ -n "$f" ] && python3 scripts/trace_list.py "$f" nx:: > $O/dec_trace_summary.txt 2>&1
f=$(find $O/prof -name "*kernel_stats.csv" | head -n 1); [ -n "$f" ] && cp "$f" $O/kernel_stats_dec_curve.csv
find $O/prof -name "*kernel_trace.csv" -delete
exit $rc
