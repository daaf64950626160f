#!/bin/bash
# Round 5 session 2: the unit-lane expander (k_expand_u) on the decode-path GPU tests, then a same-box
# timing A/B against the piece expander (NX_EXPANDER=pieces), 262 144 frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_snappy.py tests/test_gpu_decode_fuzz.py \
    tests/test_gpu_fastlz_lzf.py tests/test_gpu_lz4.py > $O/pytest_dec.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 120 python -u scripts/dec_time.py 262144 4 > $O/time_units_$i.log 2>&1 || exit 2
  NX_EXPANDER=pieces timeout -k 10 120 python -u scripts/dec_time.py 262144 4 > $O/time_pieces_$i.log 2>&1 || exit 3
done
