#!/bin/bash
# Round 5 session 8: end-to-end decode through the C-ABI batcher (bench's e2e_capi leg) with small
# batches on the fused decoder (auto) against the parse/expand pair (NX_DECODE_MODE=pair), flush-size
# sweep, and a kernel + memory-copy trace of one run for the timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s8
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
NX_SCAN_STATS=1 timeout -k 10 300 python -u scripts/long_scan_prof.py 35840 5 > $O/long_scan_stats.log 2>&1; rc=$?; echo "long_scan_stats $rc" >> $O/steps.log; fatal $rc long_scan
timeout -k 10 300 python -u scripts/long_scan_prof.py 35840 5 > $O/long_scan.log 2>&1; rc=$?; echo "long_scan $rc" >> $O/steps.log; fatal $rc long_scan
NX_HIP_DEBUG=1 timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_frame_scan.py \
    tests/test_gpu_output_staging.py > $O/pytest_staging.log 2>&1; rc=$?; echo "pytest_staging $rc" >> $O/steps.log; fatal $rc pytest_staging
export GPU_MAX_HW_QUEUES=16
for i in 1 2; do
  for mode in auto pair; do
    for fm in 256 512 1024; do
      NX_DECODE_MODE=$mode timeout -k 10 120 netty_amd/e2e_capi 256 256 65535 2 0 $fm > $O/e2e_${mode}_${fm}_$i.json 2>&1; rc=$?
      echo "e2e $mode $fm $i $rc" >> $O/steps.log; fatal $rc e2e
    done
  done
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$ROOT/$O/trace" -o tr -- \
    "$ROOT/netty_amd/e2e_capi" 256 256 65535 1 0 512 > "$ROOT/$O/trace.log" 2>&1); rc=$?; echo "trace $rc" >> $O/steps.log
unset GPU_MAX_HW_QUEUES
N=262144 timeout -k 10 700 bash scripts/pmc_alt_traffic.sh; rc=$?; echo "alt_pmc $rc" >> $O/steps.log; fatal $rc alt_pmc
mv gpurun_out/alt_traffic.json gpurun_out/alt_traffic_* $O/ 2>/dev/null
NX_HIP_DEBUG=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest_gpu $rc" >> $O/steps.log; fatal $rc pytest_gpu
exit 0
