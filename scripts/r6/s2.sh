#!/bin/bash
# Round 6 session 2: the encoder at 5 blocks per CU with the planned launches (5 x 327 680 per 100 GiB)
# and the bench's encode/decode schedule over a ring; one decode path (no NX_EXPANDER / NX_DECODE_MODE):
# whole -m gpu suite, PMC traffic (main + alt codecs) on these sources, smoke, default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6s2
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
NX_HIP_DEBUG=1 timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu $rc" >> $O/steps.log; fatal $rc pytest_gpu; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke $rc" >> $O/steps.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 bash scripts/pmc_traffic.sh; rc=$?; echo "pmc_traffic $rc" >> $O/steps.log; fatal $rc pmc
mv gpurun_out/pmc_traffic.json gpurun_out/traffic_*.log $O/ 2>/dev/null
for c in FETCH_SIZE WRITE_SIZE; do mv gpurun_out/traffic_$c $O/ 2>/dev/null; done
N=262144 timeout -k 10 400 bash scripts/pmc_alt_traffic.sh; rc=$?; echo "alt_pmc $rc" >> $O/steps.log; fatal $rc alt_pmc
mv gpurun_out/alt_traffic.json gpurun_out/alt_traffic_* $O/ 2>/dev/null
mkdir -p profiles/r06/s2 && cp $O/pmc_traffic.json $O/alt_traffic.json profiles/r06/s2/ 2>/dev/null
timeout -k 10 700 python bench.py --steps 8 --warmup 2 > $O/bench_full.log 2>&1; rc=$?; echo "bench_full $rc" >> $O/steps.log; fatal $rc bench
exit 0
