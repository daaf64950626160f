#!/bin/bash
# Round 6 closing evidence, part A (session tag $1): the whole -m gpu suite, smoke, and the PMC
# summaries the bench line reads (main traffic, issue counters, alt-codec traffic) on these sources,
# copied into profiles/r06/$1/ of this tree so that part B's bench line finds them by digest.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${1:?session tag}
O=gpurun_out/r6$T
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
NX_HIP_DEBUG=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu $rc" >> $O/steps.log; fatal $rc pytest_gpu; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke $rc" >> $O/steps.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 bash scripts/pmc_traffic.sh; rc=$?; echo "pmc_traffic $rc" >> $O/steps.log; fatal $rc pmc
mv gpurun_out/pmc_traffic.json gpurun_out/traffic_*.log $O/ 2>/dev/null
for c in FETCH_SIZE WRITE_SIZE; do rm -rf gpurun_out/traffic_$c; done
timeout -k 10 400 bash scripts/pmc_issue.sh; rc=$?; echo "pmc_issue $rc" >> $O/steps.log; fatal $rc pmc_issue
mv gpurun_out/pmc_issue.json gpurun_out/issue_*.log $O/ 2>/dev/null
for i in 1 2; do rm -rf gpurun_out/issue_$i; done
N=262144 timeout -k 10 400 bash scripts/pmc_alt_traffic.sh; rc=$?; echo "alt_pmc $rc" >> $O/steps.log; fatal $rc alt_pmc
mv gpurun_out/alt_traffic.json $O/ 2>/dev/null
rm -rf gpurun_out/alt_traffic_FETCH_SIZE gpurun_out/alt_traffic_WRITE_SIZE
exit 0
