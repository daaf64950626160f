#!/bin/bash
# Round 6 session 17: k_expand at more waves per SIMD (session 16: 24 -> 28 -> 32 waves per CU took
# k_expand 35.7 -> 35.3 -> 34.8 ms; the alt decoders up to 6.5 % faster).  All with the 2 KiB ring:
# w4b8 = session 16's best (4-wave workgroups, 8 per CU, 78 SGPRs); w8b4s = 8-wave workgroups, 4 per
# CU, SGPRs capped at 78 (32 waves, half the CRC-table copies); w6b6s = 6-wave workgroups, 6 per CU,
# 64 SGPRs (36 waves); w8b5s = 8-wave workgroups, 5 per CU, 56 SGPRs (40 waves).  SGPRs beyond the cap
# spill to VGPR lanes.  Decoder GPU tests on the three new variants, then five libraries alternated
# three times (kernel trace + alt decoders).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r6s17
mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; cp $O/../lib_product_backup17.so netty_amd/libnetty_amd.so; exit $1;; esac; }
cp netty_amd/libnetty_amd.so $O/../lib_product_backup17.so
T="tests/test_gpu_snappy.py tests/test_gpu_decode_fuzz.py tests/test_gpu_lz4.py tests/test_gpu_fastlz_lzf.py tests/test_gpu_frame_fuzz.py tests/test_gpu_frame_scan.py"
for v in w8b4s w6b6s w8b5s; do
  cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so || exit 1
  timeout -k 10 400 python -u -m pytest $T -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1; rc=$?
  echo "pytest.$v $rc" >> $O/steps.log; fatal $rc pytest$v
  [ $rc -ne 0 ] && { cp $O/../lib_product_backup17.so netty_amd/libnetty_amd.so; exit $rc; }
done
for r in 1 2 3; do
  for v in dbase w4b8 w8b4s w6b6s w8b5s; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so || exit 1
    (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/kt_${v}_$r" -o k -- \
        python3 "$ROOT/scripts/dec_curve.py" 4 262144 > "$ROOT/$O/dec_${v}_$r.log" 2>&1); rc=$?; echo "$v.$r $rc" >> $O/steps.log; fatal $rc $v
    f=$(find $O/kt_${v}_$r -name "*kernel_trace.csv" | head -n 1); [ -n "$f" ] && python3 scripts/trace_list.py "$f" k_parse k_expand > $O/trace_${v}_$r.txt
    rm -rf $O/kt_${v}_$r
    echo -n "$v " >> $O/alt_dec.log
    timeout -k 10 240 python scripts/alt_dec_time.py 262144 3 >> $O/alt_dec.log 2>&1; rc=$?; echo "alt.$v.$r $rc" >> $O/steps.log; fatal $rc alt$v
  done
done
cp $O/../lib_product_backup17.so netty_amd/libnetty_amd.so
exit 0
