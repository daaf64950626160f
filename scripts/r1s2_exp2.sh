#!/bin/bash
# encoder atomic-swap table probes: parity tests, then timing swap on/off
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_handlers.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || exit 1
for s in 1 0; do
  NX_ENC_SWAP=$s timeout -k 10 240 python scripts/prof_encode.py 262144 2 >> gpurun_out/enc_swap.log 2>&1 || exit 1
done
NX_ENC_SWAP=1 timeout -k 10 240 python scripts/prof_encode.py 1048576 2 >> gpurun_out/enc_swap.log 2>&1 || exit 1
