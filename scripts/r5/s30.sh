#!/bin/bash
# Round 5 session 30: k_parse's window with a prefetch (NX_PARSE_PF=1: each reload also loads the
# following 64 bytes into registers; a reload that moves one window forward writes them to LDS without
# a memory wait), now that the early reload makes reloads 3.5x as frequent.  base = HEAD (K = 16, no
# prefetch); pf / pf8 / pf32 = prefetch with K = 16 / 8 / 32.  Decode tests on pf first, then two
# alternations of Snappy decode under kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s30
mkdir -p $O
fatal() { cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so; case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
cp netty_amd/build_variants/libnetty_amd_pf.so netty_amd/libnetty_amd.so
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_fastlz_lzf.py \
    tests/test_gpu_batcher_alt.py tests/test_gpu_snappy.py tests/test_gpu_decode_fuzz.py > $O/pytest_pf.log 2>&1; rc=$?; echo "pytest_pf $rc" >> $O/steps.log; fatal $rc pytest_pf
[ $rc -ne 0 ] && { fatal 0 x; exit 1; }
export TMPDIR=/tmp
for r in 1 2; do
  for v in base pf pf8 pf32; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/kt_${v}_$r" -o k -- \
        python3 "$ROOT/scripts/dec_time.py" 262144 4 > "$ROOT/$O/kt_${v}_$r.log" 2>&1); rc=$?; echo "kt $v $r $rc" >> $O/steps.log; fatal $rc kt_$v
  done
done
cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so
python3 scripts/kt_summary.py $O "k_parse(" "k_parse_fastlz" "k_parse_lzf" "k_expand(" > $O/summary.jsonl 2>&1
rm -rf $O/kt_*/
exit 0
