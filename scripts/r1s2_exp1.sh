#!/bin/bash
# decode tests + decode timing + encoder table-footprint (alias) experiment
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_handlers.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || exit 1
timeout -k 10 300 python scripts/prof_decode.py 65536 3 > gpurun_out/dec_time.log 2>&1 || exit 1
for a in 0 1024 4096 16384 65536; do
  NX_ENC_ALIAS=$a timeout -k 10 240 python scripts/prof_encode.py 262144 2 >> gpurun_out/enc_alias.log 2>&1 || exit 1
done
