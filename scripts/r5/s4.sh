#!/bin/bash
# Round 5 session 4: unit expander with the period-copy fast path and literal bitmap (4 KiB ring, loads issued
# after the LDS attempts): decode tests, timing A/B against the piece expander, issue counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s4
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_snappy.py tests/test_gpu_decode_fuzz.py \
    tests/test_gpu_fastlz_lzf.py tests/test_gpu_lz4.py > $O/pytest_dec.log 2>&1; rc=$?; echo "pytest_dec $rc" >> $O/steps.log; fatal $rc pytest_dec
for i in 1 2; do
  timeout -k 10 120 python -u scripts/dec_time.py 262144 4 > $O/time_units_$i.log 2>&1; rc=$?; fatal $rc time_units
  NX_EXPANDER=pieces timeout -k 10 120 python -u scripts/dec_time.py 262144 4 > $O/time_pieces_$i.log 2>&1; rc=$?; fatal $rc time_pieces
done
N=65536 timeout -k 10 400 bash scripts/pmc_decode_lds.sh; rc=$?; echo "pmc $rc" >> $O/steps.log; fatal $rc pmc
for i in 1 2 3; do mv gpurun_out/pmcl$i $O/ 2>/dev/null; mv gpurun_out/pmcl$i.log $O/ 2>/dev/null; done
python scripts/pmc_summary.py $O/pmcl1 $O/pmcl2 $O/pmcl3 --kernel=k_expand_u > $O/pmc_k_expand_u.txt 2>&1
python scripts/pmc_summary.py $O/pmcl1 $O/pmcl2 $O/pmcl3 --kernel=k_parse > $O/pmc_k_parse.txt 2>&1
exit 0
