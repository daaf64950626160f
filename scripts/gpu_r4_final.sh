#!/bin/bash
# Round-4 closing session: the whole GPU suite, smoke, the default bench line, kernel trace and traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
bash scripts/gpu_r4_full.sh
