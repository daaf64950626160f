#!/bin/bash
# Issue counters of the bench's kernels (the decoder's real ceiling): two rocprofv3
# --pmc passes (instruction mix; wave-cycle split), each with GRBM_GUI_ACTIVE for the dispatch's cycles,
# over the same bench command as scripts/pmc_traffic.sh, summarised into gpurun_out/pmc_issue.json
# (copy it under profiles/<round>/: bench.py attaches it to roofline_decode.issue when its source
# digest matches).  At most 8 SQ counters per pass (MI355X_MICROARCH.md).
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
CHUNKS=${CHUNKS:-327680}
cd /tmp
i=0
for ctrs in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
            "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $ctrs --output-format csv -d "$ROOT/gpurun_out/issue_$i" -o p -- \
      python "$ROOT/bench.py" --total-chunks "$CHUNKS" --sub-chunks "$CHUNKS" --weak-chunks 0 --steps 1 --warmup 0 --no-latency \
      --no-probe-ceiling --no-cpu-baseline --no-e2e --no-alt --no-frame-scan > "$ROOT/gpurun_out/issue_$i.log" 2>&1 || exit 1
done
cd "$ROOT" && python scripts/pmc_issue.py gpurun_out "$CHUNKS" > gpurun_out/pmc_issue.json
