#!/bin/bash
# Round 5 session 26: k_parse reloads once 16 running lanes are out of window (NX_PARSE_RELOAD_K=16,
# now the default; s24/s25): the whole -m gpu suite, decode timing, then the main and alt-codec PMC
# traffic passes again for the changed decoder source.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s26
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
NX_HIP_DEBUG=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu $rc" >> $O/steps.log; fatal $rc pytest_gpu; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 120 python -u scripts/dec_time.py 262144 4 > $O/time_$i.log 2>&1; rc=$?; fatal $rc time; done
CHUNKS=262144 timeout -k 10 400 bash scripts/pmc_traffic.sh; rc=$?; echo "pmc_traffic $rc" >> $O/steps.log; fatal $rc pmc
mv gpurun_out/pmc_traffic.json gpurun_out/traffic_*.log $O/ 2>/dev/null
for c in FETCH_SIZE WRITE_SIZE; do mv gpurun_out/traffic_$c $O/ 2>/dev/null; done
N=262144 timeout -k 10 400 bash scripts/pmc_alt_traffic.sh; rc=$?; echo "alt_pmc $rc" >> $O/steps.log; fatal $rc alt_pmc
mv gpurun_out/alt_traffic.json gpurun_out/alt_traffic_* $O/ 2>/dev/null
exit 0
