#!/bin/bash
# Round 5 session 11: batcher spill area + per-stream DMA mirror (batcher, handler and alt-codec
# batcher tests), end-to-end at 32 / 64 MiB decode flushes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s11
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
NX_HIP_DEBUG=1 timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_batcher.py \
    tests/test_gpu_batcher_alt.py tests/test_gpu_handlers.py tests/test_gpu_pipeline.py > $O/pytest_batcher.log 2>&1; rc=$?
echo "pytest_batcher $rc" >> $O/steps.log; fatal $rc pytest_batcher; [ $rc -ne 0 ] && exit $rc
export GPU_MAX_HW_QUEUES=16
for i in 1 2; do
  for fm in 32 64; do
    timeout -k 10 120 netty_amd/e2e_capi 256 256 65535 2 0 $fm > $O/dec${fm}_$i.json 2>&1; rc=$?; echo "e2e $fm $i $rc" >> $O/steps.log; fatal $rc e2e
  done
done
exit 0
