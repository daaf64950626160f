#!/bin/bash
# Round-4 session: GPU tests of the workspace / batcher / decode paths, the e2e flush sweep, a decoder
# A/B (VARIANTS) and the per-section stamp build.  Output under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_workspace.py tests/test_gpu_batcher.py \
    tests/test_gpu_snappy.py tests/test_gpu_handlers.py tests/test_gpu_fastlz_lzf.py tests/test_gpu_lz4.py tests/test_gpu_decode_fuzz.py \
    > gpurun_out/pytest.log 2>&1 || exit 1
for f in "0 0" "0 256" "0 512" "0 1024"; do
  echo "$f" >> gpurun_out/e2e.log
  timeout -k 10 200 netty_amd/e2e_capi 256 256 65535 3 $f >> gpurun_out/e2e.log || exit 1
  echo >> gpurun_out/e2e.log
done
VARIANTS="${VARIANTS:-base0 rw2 ns12 ns14 ns16}" ROUNDS=${ROUNDS:-2} bash scripts/ab_dec.sh || exit 1
if [ -n "${CHECK_VARIANT:-}" ]; then  # the decode tests on a candidate build
  cp "netty_amd/build_variants/libnetty_amd_$CHECK_VARIANT.so" netty_amd/libnetty_amd.so || exit 1
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_snappy.py tests/test_gpu_decode_fuzz.py \
      tests/test_gpu_fastlz_lzf.py tests/test_gpu_lz4.py > gpurun_out/pytest_$CHECK_VARIANT.log 2>&1 || exit 1
fi
for v in stamps stamps16; do
  cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so || exit 1
  timeout -k 10 200 python scripts/dec_stats.py --stamps 65536 > gpurun_out/$v.json 2> gpurun_out/$v.err || exit 1
done
