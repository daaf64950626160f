#!/bin/bash
# Round 5 session 27: the early reload (burst_steps) in the FastLZ and LZF parses too.  Alt-codec
# decode tests on the working tree (cur, K = 16 everywhere), then alternating alt-codec decode timing
# (scripts/alt_dec_time.py: configs[3]'s mix) and Snappy decode timing for base (HEAD: the early
# reload in k_parse only), cur, k0 (the all-lanes rule everywhere), k8 and k32.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s27
mkdir -p $O
fatal() { cp netty_amd/build_variants/libnetty_amd_cur.so netty_amd/libnetty_amd.so; case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
cp netty_amd/build_variants/libnetty_amd_cur.so netty_amd/libnetty_amd.so
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_fastlz_lzf.py \
    tests/test_gpu_batcher_alt.py tests/test_gpu_snappy.py tests/test_gpu_decode_fuzz.py > $O/pytest_cur.log 2>&1; rc=$?; echo "pytest_cur $rc" >> $O/steps.log; fatal $rc pytest_cur
[ $rc -ne 0 ] && { fatal 0 x; exit 1; }
for r in 1 2; do
  for v in base cur k0 k8 k32; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so
    echo -n "$v " >> $O/alt.log
    timeout -k 10 200 python scripts/alt_dec_time.py >> $O/alt.log 2>&1; rc=$?; fatal $rc alt_$v
    echo -n "$v " >> $O/dec.log
    timeout -k 10 200 python scripts/dec_time.py 262144 4 >> $O/dec.log 2>&1; rc=$?; fatal $rc dec_$v
  done
done
cp netty_amd/build_variants/libnetty_amd_cur.so netty_amd/libnetty_amd.so
exit 0
