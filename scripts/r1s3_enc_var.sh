#!/bin/bash
# encoder variants (8-byte output pairs x launch-bound VGPR budget): parity + timing at 262144 chunks
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for v in ${VARIANTS:-1_6 0_6 1_8 0_8}; do
  cp netty_amd/exp/lib_$v.so netty_amd/libnetty_amd.so || exit 1
  timeout -k 10 300 python -u -m pytest tests/test_gpu_snappy.py -x -q -k encode -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/var_t_$v.log 2>&1 || exit 1
  timeout -k 10 240 python scripts/prof_encode.py 262144 2 > gpurun_out/var_$v.tmp 2>&1 || exit 1
  echo "$v $(tail -1 gpurun_out/var_t_$v.log) $(grep encode gpurun_out/var_$v.tmp)" >> gpurun_out/var.log
done
