#!/bin/bash
# Round 5 session 10: end-to-end through the C-ABI batcher — decode auto-flush sizes (64-256 MiB),
# the copied-payload upload by k_gather_host instead of one DMA copy (NX_GATHER_STAGE_MAX_MIB), and
# encode auto-flush sizes (one flush vs 512 / 1024 MiB); a trace of the 256 MiB decode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
O=gpurun_out/r5s10
mkdir -p $O
export GPU_MAX_HW_QUEUES=16
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2" >> $O/steps.log; exit $1;; esac; }
run() {  # name, env..., args
  local name=$1; shift
  timeout -k 10 120 env "$@" > $O/$name.json 2>&1; local rc=$?; echo "$name $rc" >> $O/steps.log; fatal $rc $name
}
for i in 1 2; do
  for fm in 64 128 192 256; do run dec${fm}_$i netty_amd/e2e_capi 256 256 65535 2 0 $fm; done
  run dec256_gather_$i NX_GATHER_STAGE_MAX_MIB=100000 netty_amd/e2e_capi 256 256 65535 2 0 256
  run dec128_gather_$i NX_GATHER_STAGE_MAX_MIB=100000 netty_amd/e2e_capi 256 256 65535 2 0 128
  for ef in 512 1024 2048; do run enc${ef}_$i netty_amd/e2e_capi 256 256 65535 2 $ef 256; done
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$ROOT/$O/trace" -o tr -- \
    "$ROOT/netty_amd/e2e_capi" 256 256 65535 1 1024 256 > "$ROOT/$O/trace.log" 2>&1); rc=$?; echo "trace $rc" >> $O/steps.log
exit 0
