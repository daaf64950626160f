#!/bin/bash
# Decoder PMC pass set (instructions, cycles, HBM bytes) + naive-decoder timing.
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
N=${N:-65536}
timeout -k 10 300 python scripts/prof_decode.py $N 3 > gpurun_out/dec_time.log 2>&1 || exit 1
NX_NAIVE=1 timeout -k 10 300 python scripts/prof_decode.py $N 2 >> gpurun_out/dec_time.log 2>&1 || exit 1
cd /tmp
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
            "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$ROOT/gpurun_out/pmc$i" -o p -- python "$ROOT/scripts/prof_decode.py" $N 1 > "$ROOT/gpurun_out/pmc$i.log" 2>&1 || exit 1
done
