#!/bin/bash
# Round 5 session 32: k_parse_lz4's window size (LZ4_WIN_BLOCKS: 2 / 4 (base) / 8 / 16 blocks of 16
# bytes; the parse reads byte by byte through it and reloads per lane).  LZ4 tests on z8, then two
# alternations of the alt-codec decode timing under kernel trace (configs[3]'s mix).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s32
mkdir -p $O
fatal() { cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so; case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
cp netty_amd/build_variants/libnetty_amd_z8.so netty_amd/libnetty_amd.so
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_lz4.py \
    tests/test_gpu_lz4_frame.py > $O/pytest_z8.log 2>&1; rc=$?; echo "pytest_z8 $rc" >> $O/steps.log; fatal $rc pytest_z8
[ $rc -ne 0 ] && { fatal 0 x; exit 1; }
export TMPDIR=/tmp
for r in 1 2; do
  for v in base z2 z8 z16; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/kt_${v}_$r" -o k -- \
        python3 "$ROOT/scripts/alt_dec_time.py" > "$ROOT/$O/kt_${v}_$r.log" 2>&1); rc=$?; echo "kt $v $r $rc" >> $O/steps.log; fatal $rc kt_$v
  done
done
cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so
python3 scripts/kt_summary.py $O "k_parse_lz4" "k_lz4_serial" "k_expand(" > $O/summary.jsonl 2>&1
rm -rf $O/kt_*/
exit 0
