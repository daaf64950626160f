#!/bin/bash
# HBM traffic of the bench's kernels: two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
# over one step of the bench workload (CHUNKS <= one encoder launch: every call covers all CHUNKS chunks), summarised into
# gpurun_out/pmc_traffic.json (copy it under profiles/<round>/ to back bench.py's roofline.traffic).
cd "${GRAFT_REPO_ROOT:-.}"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
CHUNKS=${CHUNKS:-327680}  # one full encoder launch on 256 CUs (round 6 plan)
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$ROOT/gpurun_out/traffic_$c" -o p -- \
      python "$ROOT/bench.py" --total-chunks "$CHUNKS" --sub-chunks "$CHUNKS" --weak-chunks 0 --steps 1 --warmup 0 --no-latency --no-probe-ceiling \
      --no-cpu-baseline --no-e2e --no-alt --no-frame-scan > "$ROOT/gpurun_out/traffic_$c.log" 2>&1 || exit 1
done
cd "$ROOT" && python scripts/pmc_traffic.py gpurun_out "$CHUNKS" > gpurun_out/pmc_traffic.json
