#!/bin/bash
# Round 5 session 17: encoder / record-expander overlap experiment (scripts/experiments/overlap.cpp).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s17
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
for sd in 16_lb5; do
  timeout -k 10 300 scripts/experiments/bin/overlap_$sd 262144 2 > $O/overlap_$sd.log 2>&1; rc=$?; echo "overlap $sd $rc" >> $O/steps.log; fatal $rc overlap
done
exit 0
