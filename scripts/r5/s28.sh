#!/bin/bash
# Round 5 session 28: kernel-trace A/B of the reload thresholds after s27 (where the FastLZ / LZF
# parses got faster from the shared step form but slower with the early reload): base (HEAD: early
# reload in all three parses, K = 16), cur (k_parse K = 16, FastLZ / LZF K = 0), k0 (K = 0 in all),
# a16 (K = 16 in all, the working tree's form).  Snappy decode (dec_time.py) and alt decode
# (alt_dec_time.py) each under rocprofv3 kernel trace, two alternations; decode tests on cur first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s28
mkdir -p $O
fatal() { cp netty_amd/build_variants/libnetty_amd_cur.so netty_amd/libnetty_amd.so; case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
cp netty_amd/build_variants/libnetty_amd_cur.so netty_amd/libnetty_amd.so
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_fastlz_lzf.py \
    tests/test_gpu_batcher_alt.py tests/test_gpu_snappy.py tests/test_gpu_decode_fuzz.py > $O/pytest_cur.log 2>&1; rc=$?; echo "pytest_cur $rc" >> $O/steps.log; fatal $rc pytest_cur
[ $rc -ne 0 ] && { fatal 0 x; exit 1; }
export TMPDIR=/tmp
for r in 1 2; do
  for v in base cur k0 a16; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/kt_${v}_$r" -o k -- \
        python3 "$ROOT/scripts/dec_time.py" 262144 4 > "$ROOT/$O/kt_${v}_$r.log" 2>&1); rc=$?; echo "kt $v $r $rc" >> $O/steps.log; fatal $rc kt_$v
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/kt_${v}alt_$r" -o k -- \
        python3 "$ROOT/scripts/alt_dec_time.py" > "$ROOT/$O/kt_${v}alt_$r.log" 2>&1); rc=$?; echo "kt ${v}alt $r $rc" >> $O/steps.log; fatal $rc kt_${v}alt
  done
done
cp netty_amd/build_variants/libnetty_amd_cur.so netty_amd/libnetty_amd.so
python3 scripts/kt_summary.py $O "k_parse(" "k_parse_fastlz" "k_parse_lzf" "k_expand(" > $O/summary.jsonl 2>&1
rm -rf $O/kt_*/
exit 0
