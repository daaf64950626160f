#!/bin/bash
# One decode A/B session: correctness of the candidate build (decode GPU tests), then alternating
# timing of the variants (scripts/ab_dec.sh).  CAND=<variant to test> VARIANTS="base cand" ROUNDS=3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp "netty_amd/build_variants/libnetty_amd_${CAND}.so" netty_amd/libnetty_amd.so || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_decode_fuzz.py tests/test_gpu_fastlz_lzf.py tests/test_gpu_lz4.py ${EXTRA_TESTS:-} -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_cand.log 2>&1 || exit 1
bash scripts/ab_dec.sh
