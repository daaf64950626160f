#!/bin/bash
# Round 5 session 12: the encoder's stream window keeps its pointer's address space (origin = in - pad
# instead of an integer mask): LDS-form reads become ds_read (were flat), HBM forms global_load (were
# flat).  Encoder tests, the placement-controlled A/B of the dense kernel (A = new, B = old), and the
# latency leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s12
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_encoder_forms.py \
    tests/test_gpu_snappy.py tests/test_gpu_output_staging.py > $O/pytest_enc.log 2>&1; rc=$?
echo "pytest_enc $rc" >> $O/steps.log; fatal $rc pytest_enc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/latency_run.py > $O/latency.log 2>&1; rc=$?; echo "latency $rc" >> $O/steps.log; fatal $rc latency
timeout -k 10 400 scripts/experiments/bin/enc_ab3_origin 262144 4 > $O/enc_ab_origin.log 2>&1; rc=$?; echo "enc_ab $rc" >> $O/steps.log; fatal $rc enc_ab
exit 0
