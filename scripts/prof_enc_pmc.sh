#!/bin/bash
# Encoder profile: kernel time (rocprofv3 --kernel-trace --stats) plus SQ instruction / wait counters,
# one --pmc pass per counter group (scripts/prof_encode.py N R runs encode only).
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); OUT=$ROOT/gpurun_out/encprof; mkdir -p "$OUT"; export TMPDIR=/tmp
N=${N:-16384}
cd /tmp
timeout -k 10 120 python "$ROOT/scripts/prof_encode.py" "$N" 2 > "$OUT/plain.log" 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- python "$ROOT/scripts/prof_encode.py" "$N" 2 > "$OUT/kt.log" 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o p -- python "$ROOT/scripts/prof_encode.py" "$N" 1 > "$OUT/pmc$i.log" 2>&1 || exit 1
done
echo done > "$OUT/done"
