#!/bin/bash
# Round 5 session 36: closing run after the host-code UBSan fix (nx::copy_bytes): the whole -m gpu suite, smoke, and the
# default bench line (now with end_to_end.link, the host link's measured budget).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s36
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
NX_HIP_DEBUG=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu $rc" >> $O/steps.log; fatal $rc pytest_gpu; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke $rc" >> $O/steps.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python bench.py > $O/bench_full.log 2>&1; rc=$?; echo "bench_full $rc" >> $O/steps.log; fatal $rc bench
exit 0
