#!/bin/bash
# Round 6 session 6: k_parse with more frames in flight.  A decode call's frames
# are k_parse's lanes, so more waves per SIMD need larger calls (NX_DEC_MAX_FRAMES = 524 288: 32 GiB of
# record slots) and, for more than 4 blocks per CU, a smaller per-lane LDS (record rows of 8 or 4:
# 6 or 7 blocks).  Library variants alternated (scripts/build_lib_variant.sh), decode + verify per call
# (scripts/dec_curve.py) at 262 144 and 524 288 frames, under a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r6s6
mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
cp netty_amd/libnetty_amd.so $O/../lib_product_backup6.so
for r in 1 2; do
  for v in dbase d524 d524q8 d524q4; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so || exit 1
    (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/kt_${v}_$r" -o k -- \
        python3 "$ROOT/scripts/dec_curve.py" 3 262144 524288 > "$ROOT/$O/dec_${v}_$r.log" 2>&1); rc=$?; echo "$v.$r $rc" >> $O/steps.log; fatal $rc $v
    f=$(find $O/kt_${v}_$r -name "*kernel_trace.csv" | head -n 1); [ -n "$f" ] && python3 scripts/trace_list.py "$f" k_parse k_expand > $O/trace_${v}_$r.txt
    rm -rf $O/kt_${v}_$r
  done
done
cp $O/../lib_product_backup6.so netty_amd/libnetty_amd.so
exit 0
