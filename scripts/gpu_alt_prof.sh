#!/bin/bash
# GPU: FastLZ / LZF / LZ4 parity tests, then a kernel-trace profile of bench.py's configs[3] leg.
# Usage (on the box): TESTS="tests/test_gpu_lz4.py ..." TAG=prof_alt bash scripts/gpu_alt_prof.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-prof_alt}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_fastlz_lzf.py tests/test_gpu_lz4.py tests/test_gpu_lz4_frame.py tests/test_gpu_handlers.py} \
    -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/$TAG" -o run -- \
    python "$ROOT/bench.py" --total-chunks 16384 --weak-chunks 0 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e \
    --no-frame-scan --no-probe-ceiling > "$ROOT/gpurun_out/$TAG/bench.log" 2>&1
