#!/bin/bash
# Round 5 session 9: k_parse with the line window (NX_PARSE_LINE=1: 128-byte line + 16-byte carry per
# reload) against the 64-byte burst window: decode tests on the line build, alternating timing, and
# FETCH_SIZE/WRITE_SIZE of both builds' kernels.  The default library is restored at the end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s9
mkdir -p $O
fatal() { cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so; case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
cp netty_amd/build_variants/libnetty_amd_line.so netty_amd/libnetty_amd.so
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_snappy.py \
    tests/test_gpu_decode_fuzz.py > $O/pytest_line.log 2>&1; rc=$?; echo "pytest_line $rc" >> $O/steps.log; fatal $rc pytest_line
[ $rc -ne 0 ] && { fatal 0 x; exit 1; }
for r in 1 2 3; do
  for v in base line; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so
    echo -n "$v " >> $O/ab.log
    timeout -k 10 200 python scripts/dec_time.py 262144 4 >> $O/ab.log 2>&1; rc=$?; fatal $rc time_$v
  done
done
export TMPDIR=/tmp
for v in base line; do
  cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$ROOT/$O/pmc_${v}_$c" -o p -- \
        python3 "$ROOT/scripts/prof_decode.py" 65536 1 > "$ROOT/$O/pmc_${v}_$c.log" 2>&1); rc=$?; echo "pmc $v $c $rc" >> $O/steps.log; fatal $rc pmc
  done
done
cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so
exit 0
