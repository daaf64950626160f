#!/bin/bash
# Round 5 session 5: the whole -m gpu suite on the round's sources (piece expander default, LZ4 HC,
# long-stream scan, small-batch fused decode), smoke, and the driver's default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s5
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu $rc" >> $O/steps.log; fatal $rc pytest_gpu; [ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke $rc" >> $O/steps.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $O/bench_full.log 2>&1; rc=$?; echo "bench_full $rc" >> $O/steps.log
exit $rc
