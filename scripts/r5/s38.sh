#!/bin/bash
# Round 5 session 38: k_parse_lz4 in burst form (LZ4_BURST=1: one lane per block as a state machine
# whose steps read at most the 5 window bytes at ip or emit one record, stepped together between
# burst reloads, early reload at K = 16 (zb) or the all-lanes rule (zb0)) against the byte-at-a-time
# parse (base = HEAD).  LZ4 tests (with the corruption fuzz) on zb and zb0, then two alternations of
# the alt-codec decode timing under kernel trace.  The variant sources: scripts/experiments/lz4_burst.patch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s38
mkdir -p $O
fatal() { cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so; case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
for v in zb zb0; do
  cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so
  timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_lz4.py \
      tests/test_gpu_lz4_frame.py tests/test_gpu_batcher_alt.py > $O/pytest_$v.log 2>&1; rc=$?; echo "pytest_$v $rc" >> $O/steps.log; fatal $rc pytest_$v
  [ $rc -ne 0 ] && { fatal 0 x; exit 1; }
done
export TMPDIR=/tmp
for r in 1 2; do
  for v in base zb zb0; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so
    (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$ROOT/$O/kt_${v}_$r" -o k -- \
        python3 "$ROOT/scripts/alt_dec_time.py" > "$ROOT/$O/kt_${v}_$r.log" 2>&1); rc=$?; echo "kt $v $r $rc" >> $O/steps.log; fatal $rc kt_$v
  done
done
cp netty_amd/build_variants/libnetty_amd_base.so netty_amd/libnetty_amd.so
python3 scripts/kt_summary.py $O "k_parse_lz4" "k_lz4_serial" "k_expand(" > $O/summary.jsonl 2>&1
rm -rf $O/kt_*/
exit 0
