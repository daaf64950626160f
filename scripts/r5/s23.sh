#!/bin/bash
# Round 5 session 23: k_parse decoding two tags per step (NX_PARSE_2TAG=1: one 16-byte window read
# serves a tag and the next when its header lies inside it) against the one-tag loop: decode tests on
# the two-tag build, alternating timing, and kernel-trace stats of both builds.  Default restored at the end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s23
mkdir -p $O
fatal() { cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so; case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
cp netty_amd/build_variants/libnetty_amd_p2tag.so netty_amd/libnetty_amd.so
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_snappy.py \
    tests/test_gpu_decode_fuzz.py > $O/pytest_p2tag.log 2>&1; rc=$?; echo "pytest_p2tag $rc" >> $O/steps.log; fatal $rc pytest_p2tag
[ $rc -ne 0 ] && { fatal 0 x; exit 1; }
for r in 1 2 3; do
  for v in base p2tag; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so
    echo -n "$v " >> $O/ab.log
    timeout -k 10 200 python scripts/dec_time.py 262144 4 >> $O/ab.log 2>&1; rc=$?; fatal $rc time_$v
  done
done
export TMPDIR=/tmp
for v in base p2tag; do
  cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/kt_$v" -o k -- \
      python3 "$ROOT/scripts/dec_time.py" 262144 4 > "$ROOT/$O/kt_$v.log" 2>&1); rc=$?; echo "kt $v $rc" >> $O/steps.log; fatal $rc kt
done
cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so
exit 0
