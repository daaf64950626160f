#!/bin/bash
# Round 5 session 21: FastLZ parse window A/B (FLZ_WIN_BLOCKS 4 / 8 / 16 = 64 / 128 / 256-byte windows)
# on the configs[3] mix, alternating library builds; the default library restored at the end.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r5s21
mkdir -p $O
cp netty_amd/libnetty_amd.so /tmp/libnetty_amd_default.so
fatal() { cp /tmp/libnetty_amd_default.so netty_amd/libnetty_amd.so; case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
for r in 1 2; do
  for v in flz4 flz8 flz16; do
    cp netty_amd/build_variants/libnetty_amd_$v.so netty_amd/libnetty_amd.so
    echo -n "$v " >> $O/ab.log
    timeout -k 10 200 python scripts/alt_dec_time.py 262144 4 2>/dev/null | tail -1 >> $O/ab.log; rc=$?; fatal $rc $v
  done
done
cp /tmp/libnetty_amd_default.so netty_amd/libnetty_amd.so
exit 0
