#!/bin/bash
# parse/expand decoder: parity tests, decode timing (auto vs fused), full bench line
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || exit 1
timeout -k 10 300 python scripts/prof_decode.py 65536 3 > gpurun_out/dec_time.log 2>&1 || exit 1
NX_VARIANT=fused timeout -k 10 300 python scripts/prof_decode.py 65536 3 >> gpurun_out/dec_time.log 2>&1 || exit 1
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/kt" -o k -- python "$GRAFT_REPO_ROOT/scripts/prof_decode.py" 65536 3 > "$GRAFT_REPO_ROOT/gpurun_out/kt.log" 2>&1 || exit 1
