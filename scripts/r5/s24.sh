#!/bin/bash
# Round 5 session 24: k_parse occupancy and record-flush variants (k_parse is LDS-limited to 4 waves
# per SIMD by its 64-byte window and 16-record queue row, 37.9 KB per 256-lane block):
#   cur   the working tree's default (= base's kernels)      q8/q4  8/4-record rows (6/7 waves per SIMD)
#   n3q8  48-byte window + 8-record rows (7 waves)           n3q4   48-byte window + 4-record rows (8 waves)
#   defer 16-record rows, the flush stored at the next put   q4d    4-record rows, deferred
#   r16   early reload: the wave reloads once 16 running lanes are out of window (not all 64)
#   r16q4 r16 + 4-record rows                                r8q4   reload at 8 + 4-record rows
# Decode tests on cur, then two alternations of decode + verify timing under rocprofv3 kernel trace
# (262 144 frames, 4 timed calls + warm-up).  Default restored at the end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s24
mkdir -p $O
fatal() { cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so; case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
cp netty_amd/build_variants/libnetty_amd_cur.so netty_amd/libnetty_amd.so
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_snappy.py \
    tests/test_gpu_decode_fuzz.py tests/test_gpu_fastlz_lzf.py tests/test_gpu_lz4.py > $O/pytest_cur.log 2>&1; rc=$?; echo "pytest_cur $rc" >> $O/steps.log; fatal $rc pytest_cur
[ $rc -ne 0 ] && { fatal 0 x; exit 1; }
export TMPDIR=/tmp
for r in 1 2; do
  for v in base cur q8 q4 n3q8 n3q4 defer q4d r16 r16q4 r8q4; do
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
