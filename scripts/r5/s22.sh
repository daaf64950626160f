#!/bin/bash
# Round 5 session 22 (bench with the in-bench oracle parity sample): the whole -m gpu suite, smoke, the driver's default bench
# line, and LZ4 HC throughput by batch size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s22
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke $rc" >> $O/steps.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python bench.py > $O/bench_full.log 2>&1; rc=$?; echo "bench_full $rc" >> $O/steps.log; fatal $rc bench
exit 0
