#!/bin/bash
# Round 5 session 18: does the encoder's throughput grow with resident lanes?  Placement-controlled
# runs (scripts/experiments/enc_ab3.cpp): A = the product kernel (32-dword stage, 4 blocks per CU),
# B = a 16-dword stage at 4 / 5 / 6 / 8 blocks per CU, each at a chunk count of one chunk per
# resident lane of B (262 144 / 327 680 / 393 216 / 524 288).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s18
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
for v in "4 262144" "5 327680" "6 393216" "8 524288"; do
  set -- $v
  timeout -k 10 300 scripts/experiments/bin/enc_ab3_s16lb$1 $2 3 > $O/enc_s16lb$1.log 2>&1; rc=$?; echo "lb$1 $rc" >> $O/steps.log; fatal $rc lb$1
done
exit 0
