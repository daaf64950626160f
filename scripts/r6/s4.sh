#!/bin/bash
# Round 6 session 4: occupancy of the alt-codec encoders (weak r5 #5).  Library variants alternated on
# one box (scripts/build_lib_variant.sh): base = FastLZ / LZF at 8 waves per CU, LZ4 at 16 (the round-5
# product); w16 = FastLZ / LZF at 16; w20 = all three at 20 waves per CU with 64-byte output stage units.
# scripts/alt_enc_time.py: the bench's configs[3] batch, encode ms per 262 144 chunks, decoded back.
# Then the Snappy encoder's launch tail: K chunks per lane in one launch against K launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r6s4
mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
cp netty_amd/libnetty_amd.so $O/../lib_product_backup.so
for r in 1 2; do
  for v in base w16 w20; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so || exit 1
    echo -n "$v " >> $O/alt_enc_ab.log
    timeout -k 10 300 python scripts/alt_enc_time.py 262144 3 >> $O/alt_enc_ab.log 2>&1; rc=$?; echo "$v.$r $rc" >> $O/steps.log; fatal $rc $v
  done
done
cp $O/../lib_product_backup.so netty_amd/libnetty_amd.so
# the tail of an encoder launch: one launch of K chunks per lane against K launches (327 680 lanes)
timeout -k 10 300 scripts/experiments/bin/enc_curve_s16lb5 2 loops 327680 1 2 5 > $O/enc_loops.log 2>&1; rc=$?; echo "enc_loops $rc" >> $O/steps.log; fatal $rc loops
exit 0
