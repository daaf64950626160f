#!/bin/bash
# parse/expand decoder: parity tests, decode timing at 64K and 256K frames, kernel trace
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_snappy.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || exit 1
timeout -k 10 300 python scripts/prof_decode.py 65536 3 > gpurun_out/dec_time.log 2>&1 || exit 1
timeout -k 10 300 python scripts/prof_decode.py 262144 3 >> gpurun_out/dec_time.log 2>&1 || exit 1
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/kt" -o k -- python "$GRAFT_REPO_ROOT/scripts/prof_decode.py" 262144 2 > "$GRAFT_REPO_ROOT/gpurun_out/kt.log" 2>&1 || exit 1
