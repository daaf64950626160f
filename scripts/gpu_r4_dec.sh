#!/bin/bash
# Round-4 decoder session: the GPU test suite on the current library, the decode PMC passes
# (scripts/pmc_decode_lds.sh), a kernel trace of a 262 144-frame decode and the stamp build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
N=65536 bash scripts/pmc_decode_lds.sh || exit 1
(export TMPDIR=/tmp; cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/kt" -o k -- \
    python "$ROOT/scripts/prof_decode.py" 262144 3 > "$ROOT/gpurun_out/kt.log" 2>&1) || exit 1
# the encoder leg alone, for the box-to-box record of the workspace placement
timeout -k 10 300 python bench.py --total-chunks 262144 --sub-chunks 262144 --weak-chunks 0 --steps 2 --warmup 1 --no-cpu-baseline \
    --no-e2e --no-alt --no-frame-scan > gpurun_out/bench_enc.log 2>&1 || exit 1
cp netty_amd/build_variants/libnetty_amd_stamps.so netty_amd/libnetty_amd.so || exit 1
timeout -k 10 200 python scripts/dec_stats.py --stamps 65536 > gpurun_out/stamps.json 2> gpurun_out/stamps.err
