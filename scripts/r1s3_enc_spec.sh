#!/bin/bash
# encoder: speculative vs in-order probe swaps — parity under both, then timing at 262144 chunks
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
NX_ENC_SPEC=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py -x -q -k "encode" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/enc_spec_t.log 2>&1 || exit 1
for s in 1 0 1 0; do
  NX_ENC_SPEC=$s timeout -k 10 240 python scripts/prof_encode.py 262144 2 > gpurun_out/enc_spec_$s.tmp 2>&1 || exit 1
  echo "spec=$s $(grep encode gpurun_out/enc_spec_$s.tmp)" >> gpurun_out/enc_spec.log
done
for w in 16 24; do
  NX_ENC_SPEC=0 NX_ENC_WAVES=$w timeout -k 10 240 python scripts/prof_encode.py 262144 2 > gpurun_out/enc_spec_w.tmp 2>&1 || exit 1
  echo "spec=0 waves=$w $(grep encode gpurun_out/enc_spec_w.tmp)" >> gpurun_out/enc_spec.log
done
