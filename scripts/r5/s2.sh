#!/bin/bash
# Round 5 session 2: the unit-lane expander (k_expand_u) on the decode-path GPU tests, a same-box timing
# A/B against the piece expander (NX_EXPANDER=pieces), then the round's new features' tests (LZ4 HC,
# maxEncodeSize / totalLength, the segmented long-stream frame walk).  A test failure does not stop
# the session; a timeout or crash (124/134/137/139) does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s2
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_snappy.py tests/test_gpu_decode_fuzz.py \
    tests/test_gpu_fastlz_lzf.py > $O/pytest_dec.log 2>&1; rc=$?; echo "pytest_dec $rc" >> $O/steps.log; fatal $rc pytest_dec
for i in 1 2; do
  timeout -k 10 120 python -u scripts/dec_time.py 262144 4 > $O/time_units_$i.log 2>&1; rc=$?; fatal $rc time_units
  NX_EXPANDER=pieces timeout -k 10 120 python -u scripts/dec_time.py 262144 4 > $O/time_pieces_$i.log 2>&1; rc=$?; fatal $rc time_pieces
done
timeout -k 10 500 python -u -m pytest -q --timeout 150 --timeout-method thread tests/test_gpu_lz4.py tests/test_gpu_lz4_frame.py \
    tests/test_gpu_frame_scan.py tests/test_gpu_handlers.py > $O/pytest_new.log 2>&1; rc=$?; echo "pytest_new $rc" >> $O/steps.log; fatal $rc pytest_new
exit 0
