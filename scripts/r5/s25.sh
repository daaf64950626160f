#!/bin/bash
# Round 5 session 25: the early-reload threshold of k_parse's tag loop (s24: reloading once 16
# running lanes are out of window, not all 64, took k_parse 12.83 -> 12.20 ms).  rK = the working tree
# (tag step as a lambda, one-compare error predicate) built with NX_PARSE_RELOAD_K=K; rKh = HEAD's tag
# loop with only the early reload added (/tmp build of scripts/build_dec_variant.sh); cur = the
# working tree's default.  Decode tests on r16h, then two alternations under kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s25
mkdir -p $O
fatal() { cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so; case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
cp netty_amd/build_variants/libnetty_amd_r16h.so netty_amd/libnetty_amd.so
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_snappy.py \
    tests/test_gpu_decode_fuzz.py tests/test_gpu_fastlz_lzf.py tests/test_gpu_lz4.py > $O/pytest_r16h.log 2>&1; rc=$?; echo "pytest_r16h $rc" >> $O/steps.log; fatal $rc pytest_r16h
[ $rc -ne 0 ] && { fatal 0 x; exit 1; }
export TMPDIR=/tmp
for r in 1 2; do
  for v in base cur r8 r12 r16 r24 r12h r16h r24h; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/kt_${v}_$r" -o k -- \
        python3 "$ROOT/scripts/dec_time.py" 262144 4 > "$ROOT/$O/kt_${v}_$r.log" 2>&1); rc=$?; echo "kt $v $r $rc" >> $O/steps.log; fatal $rc kt_$v
  done
done
cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so
# the trace databases exceed gpurun_out's 64 MiB: keep the summary and the per-kernel csv only
python3 scripts/kt_summary.py $O > $O/summary.jsonl 2>&1
python3 scripts/kt_summary.py $O "k_parse(" "k_expand(" "k_crc32c" > /dev/null 2>&1
rm -rf $O/kt_*/
exit 0
