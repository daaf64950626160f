#!/bin/bash
# Decoder candidate session: the decode-path GPU tests on the current library, then the A/B timing
# of VARIANTS (scripts/ab_dec.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_snappy.py tests/test_gpu_decode_fuzz.py \
    tests/test_gpu_fastlz_lzf.py tests/test_gpu_lz4.py tests/test_gpu_lz4_frame.py tests/test_gpu_handlers.py tests/test_gpu_frame_fuzz.py \
    tests/test_gpu_frame_scan.py tests/test_gpu_batcher.py tests/test_gpu_batcher_alt.py > gpurun_out/pytest_dec.log 2>&1 || exit 1
VARIANTS="${VARIANTS}" ROUNDS=${ROUNDS:-2} bash scripts/ab_dec.sh
