#!/bin/bash
# PMC instruction counts of decoder experiment modes (NX_DEC_MODE): one counter pass per mode
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp
N=${N:-16384}
for m in ${MODES:-0 1 2 4}; do
  NX_DEC_MODE=$m timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH --output-format csv -d "$ROOT/gpurun_out/mode$m" -o p -- python "$ROOT/scripts/prof_decode.py" $N 1 > "$ROOT/gpurun_out/mode$m.log" 2>&1 || exit 1
  NX_DEC_MODE=$m timeout -k 10 300 python "$ROOT/scripts/prof_decode.py" $N 3 >> "$ROOT/gpurun_out/mode$m.log" 2>&1 || exit 1
done
