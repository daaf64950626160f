#!/bin/bash
# Round 6 session 5: k_parse of the next piece beside k_expand of this one, on two
# streams (scripts/experiments/dec_pipe.cpp), with 128-lane parse blocks (fit beside three expander
# workgroups) and 256-lane ones (beside two), against the serial pair; 262 144 frames, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6s5
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
for b in 128 256; do
  timeout -k 10 240 scripts/experiments/bin/dec_pipe_$b 262144 2 > $O/dec_pipe_$b.log 2>&1; rc=$?; echo "pipe$b $rc" >> $O/steps.log; fatal $rc pipe$b
done
exit 0
