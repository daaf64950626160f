#!/bin/bash
# Round 5 session 6: the frame-window expander k_expand_f (NX_EXPANDER=frame): decode tests through it,
# timing A/B against the piece expander, issue counters; then the rest of the -m gpu suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s6
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
NX_EXPANDER=frame timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_snappy.py \
    tests/test_gpu_decode_fuzz.py > $O/pytest_frame.log 2>&1; rc=$?; echo "pytest_frame $rc" >> $O/steps.log; fatal $rc pytest_frame
if [ $rc -eq 0 ]; then
  for i in 1 2; do
    NX_EXPANDER=frame timeout -k 10 120 python -u scripts/dec_time.py 262144 4 > $O/time_frame_$i.log 2>&1; rc=$?; fatal $rc time_frame
    timeout -k 10 120 python -u scripts/dec_time.py 262144 4 > $O/time_pieces_$i.log 2>&1; rc=$?; fatal $rc time_pieces
  done
  NX_EXPANDER=frame N=65536 timeout -k 10 400 bash scripts/pmc_decode_lds.sh; rc=$?; echo "pmc $rc" >> $O/steps.log; fatal $rc pmc
  for i in 1 2 3; do mv gpurun_out/pmcl$i $O/ 2>/dev/null; mv gpurun_out/pmcl$i.log $O/ 2>/dev/null; done
  python scripts/pmc_summary.py $O/pmcl1 $O/pmcl2 $O/pmcl3 --kernel=k_expand_f > $O/pmc_k_expand_f.txt 2>&1
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    --deselect tests/test_gpu_snappy.py --deselect tests/test_gpu_decode_fuzz.py > $O/pytest_rest.log 2>&1
rc=$?; echo "pytest_rest $rc" >> $O/steps.log; fatal $rc pytest_rest
exit 0
