#!/bin/bash
# Round 6 session 7: the parses' tag-step control made branch-free (window test and burst predicate
# with bitwise operators; the record row written without an exec region).  Library variants alternated
# three times (dbase = before, pbf = after): Snappy decode + verify of 262 144 frames under a kernel
# trace (k_parse / k_expand per dispatch), and the alt-codec decoders (scripts/alt_dec_time.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r6s7
mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
cp netty_amd/libnetty_amd.so $O/../lib_product_backup7.so
for r in 1 2 3; do
  for v in dbase pbf; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so || exit 1
    (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/kt_${v}_$r" -o k -- \
        python3 "$ROOT/scripts/dec_curve.py" 4 262144 > "$ROOT/$O/dec_${v}_$r.log" 2>&1); rc=$?; echo "$v.$r $rc" >> $O/steps.log; fatal $rc $v
    f=$(find $O/kt_${v}_$r -name "*kernel_trace.csv" | head -n 1); [ -n "$f" ] && python3 scripts/trace_list.py "$f" k_parse k_expand > $O/trace_${v}_$r.txt
    rm -rf $O/kt_${v}_$r
    echo -n "$v " >> $O/alt_dec.log
    timeout -k 10 240 python scripts/alt_dec_time.py 262144 3 >> $O/alt_dec.log 2>&1; rc=$?; echo "alt.$v.$r $rc" >> $O/steps.log; fatal $rc alt$v
  done
done
cp $O/../lib_product_backup7.so netty_amd/libnetty_amd.so
exit 0
