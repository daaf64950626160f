#!/bin/bash
# Round 6 session 13: k_expand's instruction cuts, second step.  rdy2 = session 12's rdyasm plus the
# pass's lane masks as ballots of single compares (dependent pieces, overlapping copies; no bool
# materialised), no select of the producer range for lanes without one, and a plain round-guard exit.
# Decoder GPU tests on rdy2, then rbase / rdyasm / rdy2 alternated three times (kernel trace + alt decoders).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r6s13
mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; cp $O/../lib_product_backup13.so netty_amd/libnetty_amd.so; exit $1;; esac; }
cp netty_amd/libnetty_amd.so $O/../lib_product_backup13.so
T="tests/test_gpu_snappy.py tests/test_gpu_decode_fuzz.py tests/test_gpu_lz4.py tests/test_gpu_fastlz_lzf.py tests/test_gpu_frame_fuzz.py tests/test_gpu_frame_scan.py"
for v in rdy2; do
  cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so || exit 1
  timeout -k 10 400 python -u -m pytest $T -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1; rc=$?
  echo "pytest.$v $rc" >> $O/steps.log; fatal $rc pytest$v
  [ $rc -ne 0 ] && { cp $O/../lib_product_backup13.so netty_amd/libnetty_amd.so; exit $rc; }
done
for r in 1 2 3; do
  for v in rbase rdyasm rdy2; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so || exit 1
    (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/kt_${v}_$r" -o k -- \
        python3 "$ROOT/scripts/dec_curve.py" 4 262144 > "$ROOT/$O/dec_${v}_$r.log" 2>&1); rc=$?; echo "$v.$r $rc" >> $O/steps.log; fatal $rc $v
    f=$(find $O/kt_${v}_$r -name "*kernel_trace.csv" | head -n 1); [ -n "$f" ] && python3 scripts/trace_list.py "$f" k_parse k_expand > $O/trace_${v}_$r.txt
    rm -rf $O/kt_${v}_$r
    echo -n "$v " >> $O/alt_dec.log
    timeout -k 10 240 python scripts/alt_dec_time.py 262144 3 >> $O/alt_dec.log 2>&1; rc=$?; echo "alt.$v.$r $rc" >> $O/steps.log; fatal $rc alt$v
  done
done
cp $O/../lib_product_backup13.so netty_amd/libnetty_amd.so
exit 0
