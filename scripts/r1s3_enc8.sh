#!/bin/bash
# encoder: 8-byte candidate reads — encode parity (all align cases), then timing at 262144 chunks
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_handlers.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/enc8_t.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 240 python scripts/prof_encode.py 262144 2 >> gpurun_out/enc8.log 2>&1 || exit 1
done
