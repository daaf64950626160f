#!/bin/bash
# Round 6 session 3: the session-2 sources + weak-leg buffers freed before the extra legs, the LZ4
# encode-after-close check, HC beside-rates: PMC traffic and issue passes (the bench's call shapes),
# a kernel trace of the bench workload, and the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r6s3
mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "after_close or encoder_jobs_equal_sync or reserve_under or table_reset or ring_schedule or plan_launch" > $O/pytest_new.log 2>&1
rc=$?; echo "pytest_new $rc" >> $O/steps.log; fatal $rc pytest_new; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 bash scripts/pmc_traffic.sh; rc=$?; echo "pmc_traffic $rc" >> $O/steps.log; fatal $rc pmc
mv gpurun_out/pmc_traffic.json gpurun_out/traffic_*.log $O/ 2>/dev/null
for c in FETCH_SIZE WRITE_SIZE; do mv gpurun_out/traffic_$c $O/ 2>/dev/null; done
timeout -k 10 400 bash scripts/pmc_issue.sh; rc=$?; echo "pmc_issue $rc" >> $O/steps.log; fatal $rc pmc_issue
mv gpurun_out/pmc_issue.json gpurun_out/issue_*.log $O/ 2>/dev/null
for i in 1 2; do mv gpurun_out/issue_$i $O/ 2>/dev/null; done
mkdir -p profiles/r06/s3 && cp $O/pmc_traffic.json $O/pmc_issue.json profiles/r06/s3/ 2>/dev/null
cp gpurun_out/r6s2/alt_traffic.json profiles/r06/s3/ 2>/dev/null
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof" -o run -- \
    python3 "$ROOT/bench.py" --total-chunks 655360 --weak-chunks 0 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-alt \
    --no-frame-scan --no-latency --no-probe-ceiling > "$ROOT/$O/prof.log" 2>&1); rc=$?; echo "prof $rc" >> $O/steps.log; fatal $rc prof
f=$(find $O/prof -name "*kernel_stats.csv" | head -n 1); [ -n "$f" ] && cp "$f" $O/kernel_stats_bench.csv
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1); [ -n "$f" ] && python3 scripts/trace_list.py "$f" nx:: > $O/bench_trace_list.txt
find $O/prof -name "*kernel_trace.csv" -delete
timeout -k 10 900 python bench.py --steps 8 --warmup 2 > $O/bench_full.log 2>&1; rc=$?; echo "bench_full $rc" >> $O/steps.log; fatal $rc bench
exit 0
