#!/bin/bash
# Decode-kernel profile with the experiment harness: counters variant, kernel trace, and two SQ
# counter passes (one --pmc group per run).  BIN=dec_bench_base by default; N frames.
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); EXP=$ROOT/scripts/experiments; OUT=$ROOT/gpurun_out/decprof; mkdir -p "$OUT"; export TMPDIR=/tmp
N=${N:-65536}; BIN=${BIN:-dec_bench_base}
cd /tmp
timeout -k 10 120 "$EXP/${CBIN:-dec_bench_count}" "$N" 1 1 > "$OUT/count.log" 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- "$EXP/$BIN" "$N" 2 1 > "$OUT/kt.log" 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o p -- "$EXP/$BIN" "$N" 1 1 > "$OUT/pmc$i.log" 2>&1 || exit 1
done
echo done > "$OUT/done"
