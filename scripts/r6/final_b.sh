#!/bin/bash
# Round 6 closing evidence, part B (session tag $1; part A's PMC summaries committed under
# profiles/r06/$1/): kernel trace of the bench workload (two full encoder launches) and the default
# bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
T=${1:?session tag}
O=gpurun_out/r6$T
mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof" -o run -- \
    python3 "$ROOT/bench.py" --total-chunks 655360 --weak-chunks 0 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-alt \
    --no-frame-scan --no-latency --no-probe-ceiling > "$ROOT/$O/prof.log" 2>&1); rc=$?; echo "prof $rc" >> $O/steps.log; fatal $rc prof
f=$(find $O/prof -name "*kernel_stats.csv" | head -n 1); [ -n "$f" ] && cp "$f" $O/kernel_stats_bench.csv
f=$(find $O/prof -name "*kernel_trace.csv" | head -n 1); [ -n "$f" ] && python3 scripts/trace_list.py "$f" nx:: > $O/bench_trace_list.txt
rm -rf $O/prof
timeout -k 10 900 python bench.py --steps 8 --warmup 2 > $O/bench_full.log 2>&1; rc=$?; echo "bench_full $rc" >> $O/steps.log; fatal $rc bench
exit 0
