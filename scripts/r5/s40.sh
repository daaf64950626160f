#!/bin/bash
# Round 5 session 40: rocprofv3 kernel trace of the bench workload (262 144 chunks per dispatch) on the
# round's final kernel sources (k_parse early reload), as s14 did mid-round; keeps the stats CSV.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s40
mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof" -o run -- \
    python3 "$ROOT/bench.py" --total-chunks 262144 --weak-chunks 0 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-alt \
    --no-frame-scan --no-latency > "$ROOT/$O/prof.log" 2>&1); rc=$?; echo "prof $rc" >> $O/steps.log
f=$(find $O/prof -name "*kernel_stats.csv" | head -n 1); [ -n "$f" ] && cp "$f" $O/kernel_stats_bench_262k.csv
find $O/prof -name "*kernel_trace.csv" -delete
exit $rc
